set -eo pipefail
export TMPDIR=/tmp
# C5 flow rehearsal on a one-GPU box: 2 ranks sharing cuda:0, gloo collectives (bench.py --rehearse-one-gpu)
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --rehearse-one-gpu --steps 5 --warmup 2 --no-cpu-baseline --trajectory-csv gpurun_out/c5_traj.csv \
    > gpurun_out/c5.json 2> gpurun_out/c5.err
