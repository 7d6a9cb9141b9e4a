# c3 pass time: in-tree lib vs an alternative build ($1), alternating
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python -u tools/ws_ab.py --variants "B3=1" 2>&1 | grep "rows:" | sed "s/^/base /" || exit 1
  XPG_LIB=$1 timeout -k 10 200 python -u tools/ws_ab.py --variants "B3=1" 2>&1 | grep "rows:" | sed "s/^/alt  /" || exit 1
done
