# r1l: same-box A/B of compiler scheduling strategies on the headline decode kernel (tooling).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RUN:-r1l}
mkdir -p $OUT
for v in ${VARIANTS:-base ilp iilp lat base}; do
  if [ $v = base ]; then lib=libslatecodec.so; else lib=libslatecodec_$v.so; fi
  SLATE_LIB_VARIANT=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-host-io --no-cpu-baseline --cache /tmp/wlc > $OUT/$v.json 2> $OUT/$v.err || { echo FAIL $v; tail -5 $OUT/$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$v.json'));print('$v', d['value'], d['roofline']['kernel_ms'])"
done
