bash tools/gpu_session.sh "waves:300:python tools/xparts_waves.py"
