set -o pipefail
out=gpurun_out/r3f
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 850 python -u scripts/r3/resto_variants.py > $out/variants.jsonl 2> $out/variants.err
rc=$?
cat $out/variants.jsonl
tail -3 $out/variants.err
exit $rc
