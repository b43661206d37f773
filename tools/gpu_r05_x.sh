#!/bin/bash
set -o pipefail
for v in 1 0; do AMG_JGS_FOLD=$v timeout -k 10 120 python -u tools/debug_fold.py || exit 1; done
for v in 1 0; do AMG_JGS_FOLD=$v AMG_ATOMIC_NORET=0 timeout -k 10 120 python -u tools/debug_fold.py || exit 1; done
