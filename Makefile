# Developer entry points (the reference's Makefile:14-63, for this framework).
.PHONY: build test test-gpu lint sanitize bench bench-hub ci run clean help

PY ?= python

build: ## Compile every HIP kernel (gfx950) and the host runtime in-tree
	$(PY) -m loqa_hub_amd._native.build

test: ## CPU test tier (gloo for the multi-process paths)
	$(PY) -m pytest tests -x -q -m "not gpu"

test-gpu: ## GPU tier + smoke + bench on an MI355X box
	/usr/local/graft/bin/gpurun --timeout 1200 -- 'bash scripts/gpu_round.sh'

lint: ## Static checks (scripts/lint.py; ruff/mypy config in pyproject.toml)
	$(PY) scripts/lint.py

sanitize: ## Host runtime under ASan+UBSan and TSan (stress test)
	$(PY) -m loqa_hub_amd._native.build --sanitize address,undefined
	$(PY) -m loqa_hub_amd._native.build --sanitize thread

bench: ## Headline bench (config 4 shape, one GPU)
	$(PY) bench.py

bench-hub: ## The served path: relays over gRPC into the hub
	$(PY) bench.py --mode hub

ci: ## Everything the CPU container can run
	bash scripts/ci.sh

run: ## Serve the hub (env-configured)
	$(PY) -m loqa_hub_amd.cli.main

clean:
	rm -rf loqa_hub_amd/_native/build loqa_hub_amd/_native/*.so loqa_hub_amd/_native/*.sha256

help:
	@awk 'BEGIN {FS = ":.*?## "} /^[a-zA-Z_-]+:.*?## / {printf "  %-10s %s\n", $$1, $$2}' $(MAKEFILE_LIST)
