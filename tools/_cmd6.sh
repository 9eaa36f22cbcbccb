set -o pipefail
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gputest6.log 2>&1 || { tail -30 gpurun_out/gputest6.log; exit 1; }
tail -2 gpurun_out/gputest6.log
timeout -k 10 120 python tools/stage_times.py > gpurun_out/st6_sbu2.log 2>&1 && head -9 gpurun_out/st6_sbu2.log
DLRM_UPD_SBU=1 timeout -k 10 120 python tools/stage_times.py > gpurun_out/st6_sbu1.log 2>&1 && head -9 gpurun_out/st6_sbu1.log
timeout -k 10 200 bash tools/wave_trace.sh ops step
