#!/bin/bash
# capacity-80 variants on config 3 (tools/r03_var40.sh) and N = 20 variants at the driver's command (tools/r03_var.sh)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
bash tools/r03_var40.sh k8 k40 pc2 pc8 && bash tools/r03_var.sh head pw2
