#!/bin/bash
set -o pipefail
bash scripts/r6_pf.sh && bash scripts/r6_ab.sh
