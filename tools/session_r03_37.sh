bash tools/gpu_session.sh "slots:400:python tools/slot_sweep.py"
