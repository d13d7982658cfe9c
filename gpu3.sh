set -o pipefail
mkdir -p gpurun_out
for g in 0.25 4 32 120; do timeout -k 10 120 ./tools/gather_probe $g >> gpurun_out/probe.log 2>&1 || { echo "probe rc=$?" >> gpurun_out/probe.log; break; }; done
