# full GPU suite (post-kernel load change), scatter-only store probe, config 4 line with the
# side metrics timed back to back, and a 2-rank rehearsal of the N-GPU bench path on one GPU
bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "runprobe:200:./tools/run_probe" \
 "bench4:300:python bench.py --workload config4 --no-cpu --no-e2e" \
 "n2:300:BENCH_SHARE_GPU=1 BENCH_DIST=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu"
