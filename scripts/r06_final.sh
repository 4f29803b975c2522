#!/bin/bash
# round-6 closing pass: the GPU suite + smoke, PMC traffic (CG headline) + GAE, the kernel trace of the
# headline's command, the default bench line, C3 / C5 lines
set -e -o pipefail
cd "$(dirname "$0")/.."
bash scripts/gpu_pass.sh "$1" check pmc trace bench c3c5
