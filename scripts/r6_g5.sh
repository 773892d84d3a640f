#!/bin/bash
set -o pipefail
bash scripts/r6_dbg.sh && bash scripts/r6_fa.sh
