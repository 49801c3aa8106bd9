# Encode A/B (tooling): tools/bench_encode.py host-input legs under SLATE_ADD_PIECE / SLATE_PIN_SEGS
# modes, alternating processes; the encode GPU tests first.  usage: bash tools/enc_piece_ab.sh OUTDIR "MODES" ROUNDS
set -e
OUT=${1:-gpurun_out/pc3}; MODES=${2:-"pin0:SLATE_PIN_SEGS=0 pin1:"}; ROUNDS=${3:-2}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_encode_gpu.py tests/test_builder_device_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
for r in $(seq 1 $ROUNDS); do
  for c in none snappy; do
    for mode in $MODES; do
      name=${mode%%:*}; vars=$(echo ${mode#*:} | tr ',' ' ')
      env $vars SLATE_HOST_TRACE=1 timeout -k 10 200 python -u tools/bench_encode.py --codec $c --steps 7 > $OUT/enc_${c}_${name}_r$r.json 2> $OUT/enc_${c}_${name}_r$r.err
    done
  done
done
