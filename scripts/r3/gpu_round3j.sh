set -o pipefail
out=gpurun_out/r3j
mkdir -p $out
timeout -k 10 600 python -u scripts/r3/ipm_ab.py cocofest_amd/variants/libcfx_prev.so cocofest_amd/libcfx.so 3 > $out/ab.jsonl 2> $out/ab.err
rc=$?
cat $out/ab.jsonl
tail -3 $out/ab.err
exit $rc
