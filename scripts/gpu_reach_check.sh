set -o pipefail
O=gpurun_out/r6/reach2
mkdir -p $O
timeout -k 10 60 scripts/micro/bin/chain_bench > $O/micro.txt 2>&1 || exit 1
timeout -k 10 120 python -u -m pytest tests/test_chain_kkt.py -x -q --timeout 100 --timeout-method thread > $O/test_chain.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/reaching_warmstart.py --objectives fatigue --start reference --profile ipopt --max-iter 3000 --wall 150 --out $O/r.jsonl > $O/fat_ipopt.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/reaching_warmstart.py --objectives fatigue --start reference --profile cfx --bound-relax 1e-8 --max-iter 3000 --wall 150 --out $O/r.jsonl > $O/fat_cfx.txt 2>&1
