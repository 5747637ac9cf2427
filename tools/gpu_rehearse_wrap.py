#!/usr/bin/env python3
"""gpu_call.sh `py:` step wrapper for tools/gpu_rehearse.sh (an N-rank
bench.py rehearsal on the one-GPU box): runs it as a child process and exits
with its code.  Args: N BATCHES_PER_STEP RESIDENT (default 8 32 16)."""
import os
import subprocess
import sys

here = os.path.dirname(os.path.abspath(__file__))
args = sys.argv[1:] or ["8", "32", "16"]
sys.exit(subprocess.call(["bash", os.path.join(here, "gpu_rehearse.sh")] + args))
