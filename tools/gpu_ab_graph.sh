#!/bin/bash
# A/B: eager launches vs hipGraph capture of each run call (config-3 MLP, config-5 SGLD probes).
set -o pipefail
for a in "20" "20 graph"; do timeout -k 10 120 python tools/probe_mlp.py $a 2>&1 | tail -1; done
for a in "200" "200 graph"; do timeout -k 10 120 python tools/probe_sgld.py $a 2>&1 | tail -1; done
