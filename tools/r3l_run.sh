#!/bin/bash
# r3l: rehearsal of bench.py's N-rank path (torchrun, 2 and 4 ranks) on the one-GPU box: every rank
# on cuda:0 over gloo (SLATE_BENCH_ONE_DEVICE / SLATE_BENCH_BACKEND), configs1 and configs3 modes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/r3l}
mkdir -p $OUT
export SLATE_BENCH_ONE_DEVICE=1 SLATE_BENCH_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 1 --blocks 250000 > $OUT/n2.json 2> $OUT/n2.err || { echo N2_FAILED; tail -30 $OUT/n2.err; exit 1; }
cat $OUT/n2.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 4 --steps 5 --warmup 1 --workload configs3 --max-blocks-per-gpu 200000 > $OUT/n4c3.json 2> $OUT/n4c3.err || { echo N4_FAILED; tail -30 $OUT/n4c3.err; exit 1; }
cat $OUT/n4c3.json
