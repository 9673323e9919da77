TAG=r03q2_ab MODELS=2 VARIANTS=seg CMD="python tools/diag_sample.py" bash tools/gpu_ab.sh
