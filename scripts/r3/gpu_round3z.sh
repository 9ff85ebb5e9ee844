# The bench line with the NMPC section's solve share (no CPU legs, no MSK section).
set -o pipefail
out=gpurun_out/r3z
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --cpu-seconds 0 --no-msk > $out/bench.json 2> $out/bench.err; rc=$?
python3 -c "import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print({k: v for k, v in d['nmpc'].items() if not isinstance(v, (list, dict))})"
exit $rc
