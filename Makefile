# Build entry points (the driver uses __graft_entry__.build(); these are the
# same steps for humans and the Docker build).
PYTHON ?= python3
VERSION ?= 0.1.0

.PHONY: all native shim ops mock test test-gpu verify bench image clean

all: native

native:
	$(PYTHON) -m k8s_vgpu_scheduler_amd.utils.build all

shim:
	$(PYTHON) -m k8s_vgpu_scheduler_amd.utils.build shim

ops:
	$(PYTHON) -m k8s_vgpu_scheduler_amd.utils.build ops

mock:
	$(PYTHON) -m k8s_vgpu_scheduler_amd.utils.build mock

test:
	$(PYTHON) -m pytest tests/ -x -q -m "not gpu"

test-gpu:
	$(PYTHON) -m pytest tests/ -x -q -m gpu

verify:
	$(PYTHON) hack/verify.py all -v

bench:
	$(PYTHON) bench.py

image:
	docker build -f docker/Dockerfile -t mivgpu:$(VERSION) .

clean:
	rm -rf build k8s_vgpu_scheduler_amd/lib/*.so
