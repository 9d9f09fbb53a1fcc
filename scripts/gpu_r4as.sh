#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r4as
cd /root/repo
timeout -k 10 400 python -u scripts/probe_bert_instances.py > gpurun_out/r4as/instances.jsonl 2> gpurun_out/r4as/instances.err || { tail -20 gpurun_out/r4as/instances.err; exit 1; }
cat gpurun_out/r4as/instances.jsonl
