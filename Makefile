SHELL := /usr/bin/env bash
.SHELLFLAGS := -euo pipefail -c

.PHONY: help k8s dynamo install benchmark-env all build test test-gpu bench charts uninstall

help:
	@printf "Targets:\n"
	@printf "  k8s            single-node Kubernetes + Cilium + Prometheus (uses sudo)\n"
	@printf "  dynamo         mxserve platform (CRDs, operator) + AMD GPU operator\n"
	@printf "  install        k8s then dynamo\n"
	@printf "  charts         package the Helm charts (mxserve-crds, mxserve-platform) into dist/\n"
	@printf "  uninstall      remove the operator release (PURGE_CRDS=true: the CRDs too)\n"
	@printf "  benchmark-env  Python venv for run-benchmarks.sh\n"
	@printf "  build          compile the gfx950 HIP kernels + native runtime in-tree\n"
	@printf "  test           CPU test suite;  test-gpu: kernel/engine tests on an MI355X\n"
	@printf "  bench          headline serving benchmark (bench.py)\n"

k8s:
	sudo -E ./k8s-single-node-cilium.sh

dynamo:
	./install-dynamo-1node.sh

install: k8s dynamo

charts:
	mkdir -p dist && helm package deploy/helm/mxserve-crds deploy/helm/mxserve-platform -d dist

uninstall:
	UNINSTALL=true ./install-dynamo-1node.sh

benchmark-env:
	./setup-benchmark-env.sh

all: install

build:
	python3 setup_ext.py

test:
	python3 -m pytest tests -q -m "not gpu"

test-gpu:
	python3 -m pytest tests -q -m gpu

bench:
	python3 bench.py
