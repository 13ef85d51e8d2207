set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
NOPROF=1 bash tools/gpu_all.sh && TAG=r02a WORDS=2000000 timeout -k 10 600 bash tools/gpu_pmc2.sh > gpurun_out/pmc2_r02a.txt 2>&1; tail -60 gpurun_out/pmc2_r02a.txt
