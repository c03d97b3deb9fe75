#!/bin/bash
# diagnostics session: phase timestamps + C3 phase/grid timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools_phase_probe.py gpurun_out/probe_r1j.txt > gpurun_out/probe_r1j.log 2>&1 || exit 4
timeout -k 10 200 python tools_c3_phases.py > gpurun_out/phases_r1j.log 2>&1 || exit 5
