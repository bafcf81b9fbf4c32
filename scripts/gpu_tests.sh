export TMPDIR=/tmp
bash scripts/gpu_step.sh 600 pytest_gpu.log python -m pytest tests -m gpu -x -q || exit 1
