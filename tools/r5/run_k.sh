#!/bin/bash
# Chunk kernel ablations on this round's build: without the Suf computations, without U (timing and
# C5 instruction counts only; wrong records by design)
cd "$(dirname "$0")/../.."
PMC_CFG=c5 bash tools/r5/abl.sh r5k 2 "c5 c4" cur@cur@chunks nosuf@tools/ab/r5_nosuf@chunks nou@tools/ab/r5_nou@chunks
