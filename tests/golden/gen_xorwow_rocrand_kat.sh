#!/bin/bash
# Regenerate tests/golden/xorwow_rocrand_kat.json (needs hipcc + rocRAND headers; no GPU).
set -euo pipefail
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc -O1 -std=c++17 -o /tmp/gen_xorwow_rocrand_kat gen_xorwow_rocrand_kat.cpp
/tmp/gen_xorwow_rocrand_kat > xorwow_rocrand_kat.json
