#!/bin/bash
# loopback cache reuse: nontemporal payload loads in the 2 KiB-step emit (so
# the payload stream does not evict the wire from the Infinity Cache) plus the
# decode reading records from the end (the lines written last first) — rnt
# against HEAD (build/h3): c1 / c4, 3 rounds (outputs validated by the bench).
set -u
CASES="h3:build/h3 rnt:build/rnt" ROUNDS=3 WLS="c1" bash scripts/ab_tree.sh || exit $?
CASES="h3:build/h3 rnt:build/rnt" ROUNDS=2 WLS="c4" bash scripts/ab_tree.sh
