bash tools/gpu_session.sh "bench4:400:python bench.py --workload config4 --no-cpu"
