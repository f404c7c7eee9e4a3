# rehearsal of the driver's N>1 launch (2 ranks sharing the one GPU of this box, gloo barrier)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02z_n2.json 2> gpurun_out/r02z_n2.err
python -c "import json;d=json.loads(open('gpurun_out/r02z_n2.json').read().strip().split(chr(10))[-1]);print(d['n_gpus'], d['value'], d['ms_per_step'], d['config']['global_batch'], d['verified_frames'])"
