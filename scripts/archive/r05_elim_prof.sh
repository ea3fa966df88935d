set -o pipefail
mkdir -p gpurun_out/r05f
RLNC_LIB_PATH=$PWD/rlnc_amd/librlnc_hip_ab.so timeout -k 10 120 python scripts/elim_small_prof.py > gpurun_out/r05f/elim_prof.jsonl 2> gpurun_out/r05f/elim_prof.err || { tail gpurun_out/r05f/elim_prof.err; exit 1; }
cat gpurun_out/r05f/elim_prof.jsonl
