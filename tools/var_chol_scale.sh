set -o pipefail
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  echo "== $v"; SFM_AMD_LIB=tools/var_$v.so timeout -k 10 120 python -u tools/chol_scale.py 3000 6000 12000 || exit 1
done
