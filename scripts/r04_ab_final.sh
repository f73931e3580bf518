#!/bin/bash
# HEAD against the round-2 (87f8ae2) and round-3 (c7ff6ba) trees on c1, one box, 4 interleaved rounds.
set -u
CASES="head:. r3:build/r3 r2:build/r2" ROUNDS=4 WLS="c1" bash scripts/ab_tree.sh
