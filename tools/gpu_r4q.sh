# fp32 per-step recurrence study (r4p), then the final-build validation (r4n)
bash tools/gpu_r4p.sh || exit 1
cd $GRAFT_REPO_ROOT && bash tools/gpu_r4n.sh
