set -o pipefail
mkdir -p gpurun_out/r04i
export MV_ONLINE_DEBUG=1
echo "--- online default" 
timeout -k 5 45 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04i/smoke_default.log 2>&1; echo "rc=$?"; tail -12 gpurun_out/r04i/smoke_default.log
