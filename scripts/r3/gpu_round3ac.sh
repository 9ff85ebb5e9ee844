# cfg-5 multistart on the round-3 build (native solver, restoration phase): 64 starts at +-10 % and +-30 %, 512 at +-10 %.
set -o pipefail
out=gpurun_out/r3ac
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python3 scripts/msk_multistart_probe.py --native > $out/multistart.txt 2> $out/multistart.err; rc=$?
cat $out/multistart.txt; exit $rc
