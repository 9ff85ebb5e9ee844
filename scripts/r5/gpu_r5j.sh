# Round 5: cfg-5 512-start multistart under Ipopt's default heuristics
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
P="python3 -u scripts/msk_multistart_probe.py --native --runs 512:0.1 --jsonl $out/ms.jsonl"
timeout -k 10 150 $P --label default > $out/default.log 2>&1 || { echo "default failed"; exit 1; }
timeout -k 10 150 $P --label constant_z --opt bound_mult_init_method=constant > $out/constz.log 2>&1 || { echo "constz failed"; exit 1; }
timeout -k 10 150 $P --label filter_resets --opt max_filter_resets=5 > $out/fr.log 2>&1 || { echo "fr failed"; exit 1; }
timeout -k 10 150 $P --label ipopt_defaults --opt bound_mult_init_method=constant --opt max_filter_resets=5 --opt soft_resto_pderror_reduction_factor=0.9999 > $out/ipopt.log 2>&1 || { echo "ipopt failed"; exit 1; }
timeout -k 10 150 $P --label ipopt_defaults_maxiter3000 --max-iter 3000 --opt bound_mult_init_method=constant --opt max_filter_resets=5 --opt soft_resto_pderror_reduction_factor=0.9999 > $out/ipopt3000.log 2>&1 || { echo "ipopt3000 failed"; exit 1; }
