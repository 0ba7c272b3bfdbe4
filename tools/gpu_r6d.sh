# Round-6 step D (dev aid): cheap-half threshold A/B at 16384^2, the 4096^2
# issue variants, and the 16384^2 P=8 rank-plan issue variants.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_ab_knobs.sh t2 2 - "cheap_log2=7" "cheap_log2=6" || exit 1
N=4096 STEPS=10 bash tools/gpu_ab_knobs.sh t3 2 - "merge=1" "merge=1@--quad on" || exit 1
N=16384 P=8 bash tools/gpu_ab_sim.sh p8 1 - "merge_dist=1" "merge_dist=1@--quad on" "-@--quad on" || exit 1
