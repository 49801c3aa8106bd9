set -e
mkdir -p gpurun_out/ab/zl
for r in 1 2; do for v in zl0 zl2; do
  SLATE_LIB_VARIANT=libslatecodec_$v.so timeout -k 10 200 python -u tools/env_ab.py configs4_zstd $v: --rounds 2 > gpurun_out/ab/zl/c4_${v}_$r.txt 2>&1
done; done
for v in zl0 zl2; do SLATE_LIB_VARIANT=libslatecodec_$v.so timeout -k 10 200 python -u tools/env_ab.py kv100_zstd $v: --rounds 2 > gpurun_out/ab/zl/kv_${v}.txt 2>&1; done
