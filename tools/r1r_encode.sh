# r1r: BASELINE configs[2] encode (10 M KV) for CodecNone and Snappy, bit-exact against the oracle,
# each under a kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r1r
mkdir -p $OUT
export TMPDIR=/tmp
for c in snappy none; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $OUT/tr_$c -o run -- python3 tools/bench_encode.py --codec $c --check > $OUT/encode_$c.json 2> $OUT/encode_$c.err || { echo FAIL $c; tail -20 $OUT/encode_$c.err; exit 1; }
  cat $OUT/encode_$c.json
done
