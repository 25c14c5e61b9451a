#!/bin/bash
# Rebuild the A/B variant libraries of the current sources (tools/variants/, loaded with DREAMER_LIB_VARIANT)
# (round 6: the compile-time knobs of rounds 3-5 were removed with their untested non-default sides;
#  an A/B variant now re-adds its knob to the source first)
cd "$(dirname "$0")/.." || exit 1
rm -f tools/variants/*.so
while read -r name flags; do
  [ -z "$name" ] && continue
  python tools/build_variant.py $name $flags 2>&1 | tail -1 &
done < "${1:-tools/ab_variants.txt}"
wait
