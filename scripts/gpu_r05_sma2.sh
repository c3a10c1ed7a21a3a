cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  LIBS="dev/base.so libbt.so" CFG=5 SYMS="1250" bash scripts/gpu_ab_libs.sh || exit 1
  LIBS="dev/base.so libbt.so" CFG=2 SYMS="5000" bash scripts/gpu_ab_libs.sh || exit 1
done
