#!/bin/sh
# ref_dims.sh VARIANT IN_HEADER OUT_HEADER -- TEST INFRASTRUCTURE ONLY.
#
# Writes the reference's own ArrayLDPCMacro.h with its compile-time code dimensions substituted
# mechanically to OUT_HEADER under oracle/_ref/ (git-ignored,
# never committed, never shipped).  The reference fixes its dims by enum (ArrayLDPCMacro.h:17-39:
# MAX_ITER, the CodeWifi enum, WIDTH_MASK) and sizes the encoder's G_mlist as [972][540]
# (:196); nothing else changes.  oracle/Makefile force-includes the result ahead of the
# unmodified sources (same include guard, so the original header is then skipped).
#
#   a47r5   p47/r5 forward array code (H_array_p47_r5_forward.txt): the commented array enum at
#           :22-24, G_mlist widened to [972][1078] (max row weight of G_array_forward.txt)
#   a47r24  p47/r24 forward array code (codes/H_array_p47_r24_forward.txt): NUM_CHK 1128,
#           NUM_CGRP = VAR_DEG = 24, INFO_LENGTH 1128 (clist is sized [INFO_LENGTH], :172),
#           MAX_ITER 50, WIDTH_MASK 0x3f (BASELINE config R: 50 iterations, 6-bit mask)
set -e
variant=$1; in=$2; out=$3
case "$variant" in
  a47r5)  dims="NUM_VAR=2209 NUM_CHK=235 NUM_CGRP=5 NUM_VGRP=47 CHK_DEG=47 VAR_DEG=5 P=47 CIR_SIZE=47 INFO_LENGTH=1978 CWD_LENGTH=2209"
          extra='s/G_mlist\[972\]\[540\]/G_mlist[972][1078]/' ;;
  a47r24) dims="NUM_VAR=2209 NUM_CHK=1128 NUM_CGRP=24 NUM_VGRP=47 CHK_DEG=47 VAR_DEG=24 P=47 CIR_SIZE=47 INFO_LENGTH=1128 CWD_LENGTH=2209 MAX_ITER=50"
          extra='s/WIDTH_MASK = 0x000000ff/WIDTH_MASK = 0x0000003f/' ;;
  *) echo "ref_dims.sh: unknown variant $variant" >&2; exit 2 ;;
esac
mkdir -p "$(dirname "$out")"
script="$extra"
for kv in $dims; do
  k=${kv%%=*}; v=${kv#*=}
  script="$script
s/\\b$k = [0-9]*/$k = $v/g"
done
sed -e "$script" "$in" > "$out.tmp"
# every substitution must have taken effect on the live (uncommented) enum lines
for kv in $dims; do
  k=${kv%%=*}; v=${kv#*=}
  grep -v '^[[:space:]]*//' "$out.tmp" | grep -Eq "\\b$k = $v\\b" || { echo "ref_dims.sh: $k not set" >&2; exit 1; }
done
case "$variant" in
  a47r5)  grep -q 'G_mlist\[972\]\[1078\]' "$out.tmp" ;;
  a47r24) grep -q 'WIDTH_MASK = 0x0000003f' "$out.tmp" ;;
esac
mv "$out.tmp" "$out"
