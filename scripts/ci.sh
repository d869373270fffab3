#!/bin/bash
# CI for the CPU container (the reference's .github/workflows/ci.yml:17-71:
# build, race-enabled tests, vet / staticcheck). Stages:
#   1. native build: every HIP kernel for gfx950 + the host runtime (hipcc
#      cross-compiles without a GPU), then the package imports
#   2. lint: scripts/lint.py (+ ruff / mypy when installed)
#   3. host sanitizers: the C++ runtime (KV block pool, PCM stager, TP control
#      ring) under ASan+UBSan and under TSan with a multi-threaded stress test
#      (the `go test -race` role)
#   4. CPU test tier: pytest -m "not gpu" (multi-process paths over gloo)
# The GPU tier runs on an MI355X: scripts/gpu_round.sh (through gpurun).
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
step() { echo; echo "=== $*"; }

step "native build (gfx950)"
python -c "import __graft_entry__ as g; g.build()"

step "lint"
python scripts/lint.py
if python -c "import ruff" 2>/dev/null || command -v ruff >/dev/null; then ruff check .; fi
if python -c "import mypy" 2>/dev/null; then python -m mypy; fi

step "host sanitizers (ASan+UBSan, TSan)"
python -m loqa_hub_amd._native.build --sanitize address,undefined
python -m loqa_hub_amd._native.build --sanitize thread

step "CPU tests"
python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider ${PYTEST_ARGS:-}
echo; echo "ci: all stages passed"
