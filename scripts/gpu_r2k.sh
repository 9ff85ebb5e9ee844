# Native interior point after the watchdog / safe-slack changes: parity tests, then wall-clock probes.
set -o pipefail
out=gpurun_out/r2k
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --tb=short --timeout 300 --timeout-method thread tests/test_ipm_native.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 300 python3 scripts/profile_msk_native.py 1 64 > $out/msk.json 2> $out/msk.err || { tail -20 $out/msk.err; exit 1; }
cat $out/msk.json
timeout -k 10 300 python3 scripts/ipm_native_probe.py > $out/probe.json 2> $out/probe.err || { tail -20 $out/probe.err; exit 1; }
cat $out/probe.json
