# the driver's launch form at N = 1 (torch.distributed.run, one rank, RCCL world of 1)
set -o pipefail
mkdir -p gpurun_out/r06al
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 1 --steps 5 --warmup 2 --cpu-seconds 0 --pdsch-steps 5 --pdsch-low-snr 0 > gpurun_out/r06al/torchrun1.json 2> gpurun_out/r06al/torchrun1.err \
  || { tail -20 gpurun_out/r06al/torchrun1.err; exit 1; }
python tools/bench_brief.py gpurun_out/r06al/torchrun1.json
