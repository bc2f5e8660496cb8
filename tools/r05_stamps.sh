cd $GRAFT_REPO_ROOT || exit 2
mkdir -p gpurun_out/r05
N_ENVS=65536 GS=8 timeout -k 10 150 python tools/stamps.py > gpurun_out/r05/stamps_c3.log 2>&1 || { tail -5 gpurun_out/r05/stamps_c3.log; exit 1; }
cat gpurun_out/r05/stamps_c3.log
N_ENVS=65536 GS=16 AGENTS=4 ZOMBIES=20 timeout -k 10 150 python tools/stamps.py > gpurun_out/r05/stamps_c5.log 2>&1 || { tail -5 gpurun_out/r05/stamps_c5.log; exit 1; }
cat gpurun_out/r05/stamps_c5.log
N_ENVS=8192 GS=16 timeout -k 10 150 python tools/stamps.py > gpurun_out/r05/stamps_n8.log 2>&1 || { tail -5 gpurun_out/r05/stamps_n8.log; exit 1; }
cat gpurun_out/r05/stamps_n8.log
