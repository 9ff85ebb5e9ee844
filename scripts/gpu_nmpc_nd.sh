# NMPC (cfg 4, 64 scenarios) wall-clock with nested dissection allowed at batch 64 (CFX_IPM_ND_BATCH) and P parts.
set -o pipefail
o=gpurun_out/nmpc_nd; mkdir -p $o
run() { tag=$1; shift; timeout -k 10 300 env "$@" python -u bench.py --steps 5 --warmup 2 --batch 65536 --cpu-seconds 0 --no-msk --nmpc-horizons 100 > $o/$tag.json 2> $o/$tag.err || exit 1; }
run base CFX_IPM_ND_BATCH=8
run nd8 CFX_IPM_ND_BATCH=64 CFX_IPM_PARTS=8
run nd4 CFX_IPM_ND_BATCH=64 CFX_IPM_PARTS=4
run nd2 CFX_IPM_ND_BATCH=64 CFX_IPM_PARTS=2
run nd16 CFX_IPM_ND_BATCH=64 CFX_IPM_PARTS=16
