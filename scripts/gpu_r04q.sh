#!/bin/bash
# round 4: r04o (full suite + profiled bench + CSV recompute), then r04p (per-op timings + PMC traffic)
TAG=${TAG:-r04q} bash scripts/gpu_r04o.sh || exit 1
TAG=${TAG:-r04q}_p bash scripts/gpu_r04p.sh || exit 1
