#!/bin/bash
# Coverage-guided fuzzing of the C .ot reader (oaz_ot_read) under AddressSanitizer + UBSan, on the
# host (no GPU). Seeds: .ot files written by onitama_az.weights.write_ot (trained 3-block, random
# 0- and 1-block networks), one written by the C writer (oaz_ot_write), and archives whose data.pkl
# aliases containers through the memo (self-append, a 64-level doubling DAG, a 100 000-deep chain,
# a two-list cycle: the inputs of tests/test_host.py test_ot_readers_bounded_on_crafted_pickles).
#   tools/ot_fuzz.sh [seconds=120] [workers=4]
set -euo pipefail
cd "$(dirname "$0")/.."
SECS=${1:-120}
JOBS=${2:-4}
OUT=${OT_FUZZ_DIR:-/tmp/ot_fuzz}
mkdir -p "$OUT/corpus" "$OUT/seed"
CSRC=onitama-alphazero_amd/csrc
# plain host clang (no offload target: the reader is host code; hip_runtime.h only for its types)
/opt/rocm/lib/llvm/bin/clang++ -O1 -g -std=c++17 -fsanitize=fuzzer,address,undefined \
    -fno-sanitize-recover=undefined -mllvm -asan-globals=0 -D__HIP_PLATFORM_AMD__=1 -I /opt/rocm/include -I include \
    tools/ot_fuzz.cpp $CSRC/oaz_weights_io.cpp -o "$OUT/ot_fuzz"
PYTHONPATH=onitama-alphazero_amd python3 - "$OUT/seed" <<'EOF'
import sys
import numpy as np
from onitama_az import weights as W
d = sys.argv[1]
W.write_ot(f"{d}/trained3.ot", W.named_from_blob(np.load("tests/golden/weights_3block_trained.npy"), 3))
for b in (0, 1):
    W.write_ot(f"{d}/random{b}.ot", W.named_from_blob(W.random_weights(b, b), b))
W.save_blob_ot(f"{d}/c_writer2.ot", W.random_weights(2, 2), 2)
crafted = {
    "self_append": b"\x80\x02]q\x00h\x00ah\x00a.",
    "doubling_dag": b"\x80\x02]r\x00\x00\x00\x00" + b"".join(
        b"]r" + k.to_bytes(4, "little") + (b"j" + (k - 1).to_bytes(4, "little") + b"a") * 2 for k in range(1, 65)) + b".",
    "deep_chain": b"\x80\x02" + b"]" * 100_000 + b"a" * 99_999 + b".",
    "two_cycle": b"\x80\x02]q\x00]q\x01h\x00ah\x01a.",
}
for name, pkl in crafted.items():
    z = W._AlignedZip(f"{d}/{name}.ot")
    z.add("m/data.pkl", pkl)
    z.close()
EOF
# (libFuzzer writes its per-worker fuzz-<n>.log into the working directory)
cd "$OUT"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1:detect_odr_violation=0 UBSAN_OPTIONS=print_stacktrace=1 \
    "$OUT/ot_fuzz" "$OUT/corpus" "$OUT/seed" -max_total_time="$SECS" -jobs="$JOBS" -workers="$JOBS" \
    -max_len=400000 -rss_limit_mb=4096 -artifact_prefix="$OUT/" 2>&1 | tail -n 30
ls "$OUT"/crash-* "$OUT"/leak-* "$OUT"/timeout-* 2>/dev/null && exit 1
echo "ot_fuzz: no crash, leak or timeout in ${SECS}s x ${JOBS} workers"
