#!/usr/bin/env bash
# Node GPU inventory (replaces the Swarm node labels of reference scripts/setup_node.sh): count the
# MI355X GPUs visible to ROCm and print the value to export as RAFIKI_GPUS_PER_NODE.
set -euo pipefail
n=$(python -c "import torch; print(torch.cuda.device_count())" 2>/dev/null || echo 0)
echo "export RAFIKI_GPUS_PER_NODE=$n"
