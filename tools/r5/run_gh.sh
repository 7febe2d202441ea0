#!/bin/bash
# run_g (regroup in place: tests, A/B, kernel stats) then run_h (histogram packing with one dead shard)
cd "$(dirname "$0")/../.."
bash tools/r5/run_g.sh && bash tools/r5/run_h.sh
