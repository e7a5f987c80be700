bash tools/gpu_session.sh "waves:300:WAVES_C3=1 python tools/xparts_waves.py"
