# same-box A/B of several builds of the library (genome_graph_annotation_amd/_ab/lib*.so, in-tree last),
# alternating, Kingsford shape; usage: bash tools/gpu/ab_multi.sh [variants]
set -o pipefail
mkdir -p gpurun_out
V=${1:-0}
for r in 1 2; do
  for L in genome_graph_annotation_amd/_ab/lib*.so; do
    n=$(basename $L .so)
    MBRWT_LIB=$L timeout -k 10 300 python -u tools/sweep.py --variants $V --reps 3 > gpurun_out/abm_${n}_$r.log 2>&1 || exit 1
  done
  timeout -k 10 300 python -u tools/sweep.py --variants $V --reps 3 > gpurun_out/abm_intree_$r.log 2>&1 || exit 1
done
