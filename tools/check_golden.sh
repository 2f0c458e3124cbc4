#!/bin/bash
# Regenerate the golden fixtures from the reference into a scratch directory and compare
# them byte for byte with tests/golden/ (needs /root/reference; never runs on the GPU box).
set -e
cd "$(dirname "$0")/.."
out=$(mktemp -d)
python tools/gen_golden.py --out "$out" > "$out/gen.log"
status=0
for f in tests/golden/*.npz; do
  b=$(basename "$f")
  if cmp -s "$f" "$out/$b"; then echo "same     $b"; else echo "DIFFERS  $b"; status=1; fi
done
rm -rf "$out"
exit $status
