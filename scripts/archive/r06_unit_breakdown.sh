# round 6: per-term breakdown of the 8-wave encode unit at head (VERDICT r05 "Next round" 3).  Timing-only builds
# of the shipped 8-wave program with one term removed each (gen_bsjump.py --diag=s8*, built by scripts/bsj_diag.sh
# into build/diag_<name>/), interleaved with the product library by scripts/sweep.py (the bench's encode launch:
# 32 objects x 32 x 1 MiB -> 64 coded pieces, variant 8; the 32-row "dec" product is the 4-wave program, unchanged
# by these flags: a control).  Two interleaved passes.
set -o pipefail
O=${1:-gpurun_out/r06_unit}
mkdir -p $O
for rep in 1 2; do
  for d in product ${DIAGS:-s8inline s8noread s8noown s8nosmem s8nobar s8nodma s8nostage}; do
    if [ $d = product ]; then unset RLNC_LIB_PATH; else export RLNC_LIB_PATH=$PWD/build/diag_$d/librlnc_hip.so; fi
    echo "== $d rep $rep" >> $O/sweep.txt
    RLNC_DIAG=1 timeout -k 10 120 python scripts/sweep.py --objects 32 --configs 8:0 --rounds ${ROUNDS:-12} >> $O/sweep.txt 2>&1 || { tail $O/sweep.txt; exit 1; }
  done
done
cat $O/sweep.txt
