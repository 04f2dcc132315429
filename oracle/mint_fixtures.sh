#!/bin/bash
# TEST INFRASTRUCTURE ONLY: mints tests/golden/ref/ with the UNMODIFIED reference (oracle/_ref/ref_harness,
# built by `make -C oracle ref` from /root/reference/include). Every command is deterministic (the
# harness interposes getrandom with a seeded splitmix64 stream), so re-running reproduces the files.
#   ./oracle/mint_fixtures.sh [out-dir]        (default tests/golden/ref)
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${1:-$ROOT/tests/golden/ref}"
H="$ROOT/oracle/_ref/ref_harness"
make -C "$ROOT/oracle" ref
mkdir -p "$OUT"
"$H" fp "$OUT"                 # Fp vectors incl. non-canonical edge cases
"$H" fixtures "$OUT" 8 3 2     # 8 fresh pairs (add/sub/mul + streams), chain x fresh steps 1-3, squares 1-2
"$H" enc "$OUT" 12             # secret key, PRF vectors, 12 enc_value outputs with their streams
"$H" encdepth "$OUT"           # enc_value_depth / enc_zero_depth, depth hints 1-15
"$H" encdeep "$OUT"            # depth hints 16-100, non-default noise Params
"$H" fullrange "$OUT"          # ct_mul with weights anywhere in [0, 2^128)
"$H" chainx "$OUT" 4           # chain entry point: x = enc_value(2), c_k = ct_mul(c_{k-1}, x), k <= 4, full stream
"$H" chainf "$OUT" 4           # the reference's own loop: a fresh enc_value(2) operand per step, k <= 4, full stream
"$H" chainf8 "$OUT" 8          # the same loop to depth 8: per-step commit digests, stream stretches (manifest only)
