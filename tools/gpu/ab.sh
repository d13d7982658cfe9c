# Same-box A/B of the traversal kernel: the in-tree library vs a saved build
# (MBRWT_LIB=genome_graph_annotation_amd/_ab/libmbrwt_base.so), alternating, Kingsford shape
set -o pipefail
mkdir -p gpurun_out
BASE=genome_graph_annotation_amd/_ab/libmbrwt_base.so
for r in 1 2; do
  MBRWT_LIB=$BASE timeout -k 10 300 python -u tools/sweep.py --variants 0 --reps 3 > gpurun_out/ab_base_$r.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/sweep.py --variants 0 --reps 3 > gpurun_out/ab_new_$r.log 2>&1 || exit 1
done
