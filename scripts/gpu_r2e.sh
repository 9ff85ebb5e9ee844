# Round 2: kernel trace of the native interior point at batch 1 (cfg 3, cfg 2, cfg 5 RK4 x 5).
set -o pipefail
mkdir -p gpurun_out/ipmprof
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ipmprof -o run -- python3 scripts/ipm_native_probe.py native > gpurun_out/ipmprof/probe.json 2> gpurun_out/ipmprof/probe.err
rc=$?; cat gpurun_out/ipmprof/probe.json; find gpurun_out/ipmprof -name "*kernel_stats.csv" | head; exit $rc
