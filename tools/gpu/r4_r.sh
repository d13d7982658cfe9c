# r04 step R: where the wire's unpack time goes (kernel trace of the wire
# micro-benchmark)
set -o pipefail
mkdir -p gpurun_out/r4r
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4r/prof -o wire --output-format csv -- python3 tools/bench_wire.py > gpurun_out/r4r/bench_wire_prof.log 2>&1 || exit 1
