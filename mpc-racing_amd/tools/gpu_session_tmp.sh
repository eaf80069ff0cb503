set -u
mkdir -p gpurun_out
bash mpc-racing_amd/tools/gpu_flags_ab.sh pair nopair nopair464
