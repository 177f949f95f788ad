#!/usr/bin/env python3
"""Run one gpurun call, retrying ONLY when the infrastructure failed before the command ran
(transient box preparation / back-off / no box free).  A command that ran is never retried."""
import json
import os
import subprocess
import sys
import time

GPURUN = "/usr/local/graft/bin/gpurun"
LAST = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", ".last_call.json")


def main():
    timeout = sys.argv[1]
    cmd = sys.argv[2]
    for attempt in range(8):
        try:
            os.remove(LAST)
        except OSError:
            pass
        p = subprocess.run([GPURUN, "--timeout", timeout, "--", cmd], capture_output=True, text=True)
        out = p.stdout + p.stderr
        ran = False
        try:
            d = json.load(open(LAST))
            ran = d.get("status") not in ("transient",) and d.get("run_s", 0) > 0
        except Exception:
            d = {}
        backoff = ("backing off" in out or "stopped responding" in out or "; retry" in out
                   or p.returncode == 3 or d.get("status") == "transient")
        if ran or not backoff:
            print(out[-3000:])
            return p.returncode
        print(f"[gpu.py] infra not ready (attempt {attempt + 1}): {out.strip()[-200:]}", flush=True)
        time.sleep(30 + 15 * attempt)
    print(out[-3000:])
    return 1


if __name__ == "__main__":
    sys.exit(main())
