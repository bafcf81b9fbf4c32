# Build / test entry points with the reference's shape (/root/reference/src/Makefile:26,43:
# `make all` builds master, worker, file_server; `make clean`).  Here the three roles are
# Python entry points over native code, so `all` builds the native code in-tree:
#   serverless_learn_amd/_native/libslkernels.so   every HIP kernel, hipcc --offload-arch=gfx950
#   serverless_learn_amd/_native/_slcore*.so       C++ runtime core (wire codec, membership, ingest)
PYTHON ?= python3

.PHONY: all kernels core clean test test-gpu sanitize bench roles

all:
	$(PYTHON) -m serverless_learn_amd.build

kernels:
	$(PYTHON) -m serverless_learn_amd.build --only kernels

core:
	$(PYTHON) -m serverless_learn_amd.build --only core

test: all
	$(PYTHON) -m pytest tests -q -m "not gpu"

test-gpu: all
	$(PYTHON) -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread

sanitize:
	bash scripts/sanitize_core.sh

bench: all
	$(PYTHON) bench.py

# the reference's three processes on one host (master :50052, file server :50053)
roles:
	@echo "$(PYTHON) -m serverless_learn_amd.cli file-server"
	@echo "$(PYTHON) -m serverless_learn_amd.cli master"
	@echo "$(PYTHON) -m serverless_learn_amd.cli worker localhost:50061"

clean:
	rm -rf build serverless_learn_amd/_native/*.so serverless_learn_amd/_native/variants
