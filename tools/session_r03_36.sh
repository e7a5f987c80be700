# verify_files on the verdict: full GPU suite, then config 4 with its e2e legs
bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "bench4:400:python bench.py --workload config4 --no-cpu"
