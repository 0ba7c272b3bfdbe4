# Round-6 step F (dev aid): quad_update workgroup size A/B (16384^2, 4096^2),
# the P=8 rank plan on the current build, a 4096^2 kernel profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_ab_knobs.sh t4 2 - "upd_threads=512" || exit 1
N=4096 STEPS=10 bash tools/gpu_ab_knobs.sh t5 2 - "upd_threads=512" || exit 1
N=16384 P=8 bash tools/gpu_ab_sim.sh p8b 1 - || exit 1
timeout -k 10 300 bash tools/gpu_prof.sh 4096 bf16x6 || exit 1
