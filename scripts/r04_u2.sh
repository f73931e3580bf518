#!/bin/bash
# configs[3]: the long-payload instance with 2 KiB consumer steps (u2nt)
# against HEAD's 1 KiB steps (h2), both with nontemporal payload loads; 3 rounds.
set -u
CASES="h2:build/h2 u2nt:build/u2nt" ROUNDS=3 WLS="c3" bash scripts/ab_tree.sh
rc=$?; [ $rc = 0 ] || exit $rc
# decode window loads nontemporal (dnt) against HEAD: c3 / c1 / c2, 3 rounds
CASES="h2:build/h2 dnt:build/dnt" ROUNDS=3 WLS="c3 c1 c2" bash scripts/ab_tree.sh
