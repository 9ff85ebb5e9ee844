# 2-rank rehearsal of the multi-GPU bench on one card (gloo backend, both ranks on cuda:0): every section that runs on
# all ranks (cfg-2 headline, cfg-5 MSK, cfg-4 NMPC with the final all-gather), max-over-ranks timing.
set -o pipefail
out=gpurun_out/gloo2
mkdir -p $out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo --nmpc-horizons 20 > $out/bench.json 2> $out/bench.err; rc=$?
tail -c 600 $out/bench.json; exit $rc
