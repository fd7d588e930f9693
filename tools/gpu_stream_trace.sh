# timeline of the pinned-input verify path (kernel + memory-copy trace)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MV_STREAM_BATCHES=2 timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/tl -o run -f csv -- python tools/pipe_probe.py > gpurun_out/tl.log 2>&1 || exit 1
python tools/timeline.py gpurun_out/tl 9 > gpurun_out/timeline.txt
head -c 200 gpurun_out/timeline.txt
