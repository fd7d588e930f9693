# Rehearsal of the multi-rank bench on a 1-GPU box: 2 ranks share GPU 0 (reduced sizes), then
# the default line at N=1 for comparison of the JSON shape.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 10 --warmup 2 --batch 262144 --config4-batch 65536 --wal-entries 65536 --cpu-sample 65536 \
  --sustain-repeats 2 --sustain-seconds 0.5 > gpurun_out/ranks2.json 2> gpurun_out/ranks2.err || { tail -20 gpurun_out/ranks2.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/ranks2.json')); print(d['n_gpus'], round(d['value']/1e6,1), d['correct'], d['config']['parallelism'], round(d['config4']['value']/1e6,1), d['wal']['value'], d['scaling'])"
