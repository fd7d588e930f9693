set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_blocks.py -m gpu -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1
bash tools/ab.sh regpf main regpf main || exit 1
C2="python bench.py --steps 5 --warmup 1 --cpu-sample 0 --no-e2e --sustain-repeats 0 --no-adversarial --no-config4 --no-wal --streams 1"
OUT=gpurun_out/pb
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1 -o run -- $C2 > $OUT/t.log 2>&1 || exit 1
i=0
for g in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES"; do i=$((i+1)); timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d $OUT/pmc$i -o run -- $C2 > $OUT/p$i.log 2>&1 || exit 1; done
python tools/pmc_summary.py $OUT k_bv_bucket --json $OUT/pmc_c2_k_bv_bucket.json | tail -10
