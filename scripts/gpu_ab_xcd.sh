# XCD block mapping at head: runs of 16 blocks per XCD (head) against one contiguous range per XCD and runs
# of 64 / 128, from rest and mid-collapse (interleaved A/B).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash scripts/variant_ab.sh "head x0 x64 x128" 3
