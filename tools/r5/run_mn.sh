#!/bin/bash
cd "$(dirname "$0")/../.."
bash tools/r5/run_m.sh && bash tools/r5/run_n.sh
