# A/B of the headline launch: current library vs variant builds (CFX_LIB), launch-shape sweep.
set -o pipefail
o=gpurun_out/store_probe.jsonl; : > $o
run() { timeout -k 10 120 env "$@" python -u scripts/store_probe.py >> $o 2> gpurun_out/store_probe.err || exit 1; }
L=var_libs/libcfx_ldnt.so
for rep in 1 2; do run CFX_LIB=cocofest_amd/libcfx.so; run CFX_LIB=$L; done
for k in 3 5; do run CFX_KPT=$k; run CFX_KPT=$k CFX_LIB=$L; done
cat $o
