#!/bin/bash
# Regenerate tests/golden/map_small/ (map.cereal, opt_calib.json, expect.bin) with oracle/_ref/map_writer — the
# reference's vendored cereal writing a synthetic stereo map (oracle/map_writer.cpp).  Build container only.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
make -s -C "$ROOT/oracle" _ref/map_writer
test -x "$ROOT/oracle/_ref/map_writer" || { echo "reference not present"; exit 1; }
"$ROOT/oracle/_ref/map_writer" "$ROOT/tests/golden/map_small" 10 300 42
