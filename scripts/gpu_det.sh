export TMPDIR=/tmp
bash scripts/gpu_step.sh 300 det.log python scripts/debug_determinism.py || exit 1
