# cfg-3 multi-start solves with nested dissection allowed at larger batches (CFX_IPM_ND_BATCH; 2 blocks each).
set -o pipefail
o=gpurun_out/cfg3_nd; mkdir -p $o
run() { tag=$1; shift; timeout -k 10 300 env "$@" python -u bench.py --steps 5 --warmup 2 --batch 65536 --cpu-seconds 0 --no-msk --nmpc-horizons 0 > $o/$tag.json 2> $o/$tag.err || exit 1; }
run base CFX_IPM_ND_BATCH=64
run nd4096 CFX_IPM_ND_BATCH=4096
run base2 CFX_IPM_ND_BATCH=64
