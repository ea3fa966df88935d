set -u
cd $GRAFT_REPO_ROOT
for d in product novm nosmem novm_nosmem; do
  if [ $d = product ]; then unset RLNC_LIB_PATH; else export RLNC_LIB_PATH=build/diag_$d/librlnc_hip.so; fi
  echo "== $d"
  RLNC_DIAG=1 timeout -k 10 120 python scripts/sweep.py --configs 5:0 --rounds 10 || exit $?
done
