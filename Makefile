# Build, test and verify targets (the reference Makefile:43-129 analog).
# No network is assumed: every target uses the tools already in the image.
IMAGE_REPO ?= registry.local/xsched-amd
IMAGE_TAG ?= 0.3.0
PYTHON ?= python3
GPURUN ?= /usr/local/graft/bin/gpurun

.PHONY: all build build-core build-hip native-tests test test-gpu verify crds image bench bench-remote clean

all: build

build: build-core build-hip

build-core:
	$(PYTHON) -m flex_gpu_scheduler_amd.build_ext --core

build-hip:
	PYTORCH_ROCM_ARCH=gfx950 $(PYTHON) -m flex_gpu_scheduler_amd.build_ext --hip

native-tests:
	$(PYTHON) -m flex_gpu_scheduler_amd.build_ext --tests

# CPU tier (what CI runs here); the GPU tier needs an MI355X.
test: build-core
	$(PYTHON) -m pytest tests/ -x -q -m "not gpu"

test-gpu:
	$(PYTHON) -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread

# Lint (Python AST + text checks, C++/HIP text checks), CRD regeneration
# diff, chart rendering and image references, example configs, Dockerfile.
verify:
	$(PYTHON) -m flex_gpu_scheduler_amd.tools.verify

crds:
	$(PYTHON) -m flex_gpu_scheduler_amd.deploy.crds deploy/crds

image:
	docker build -f deploy/docker/Dockerfile -t $(IMAGE_REPO):$(IMAGE_TAG) .

bench:
	$(PYTHON) bench.py

bench-remote:
	$(PYTHON) -m flex_gpu_scheduler_amd.tools.remote_bench --matrix

clean:
	rm -rf build
