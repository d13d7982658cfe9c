set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for g in 4 32 118 200; do
timeout -k 10 200 python tools/probe_sweep.py --gib $g --segs 64 --out gpurun_out/tlb_$g.json > gpurun_out/tlb_$g.log 2>&1 || exit 1
done
