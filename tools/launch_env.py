"""Launch + completion latency of the bench window under HIP runtime settings (each in a fresh
process, since the runtime reads them at init): tools/launch_cost.py --quick per setting.

    python tools/launch_env.py
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SETTINGS = [
    {},
    {"HIP_FORCE_DEV_KERNARG": "1"},
    {"ROC_ACTIVE_WAIT_TIMEOUT": "100"},
    {"HIP_FORCE_DEV_KERNARG": "1", "ROC_ACTIVE_WAIT_TIMEOUT": "100"},
    {"HIP_FORCE_DEV_KERNARG": "1", "ROC_ACTIVE_WAIT_TIMEOUT": "100", "ROC_CPU_WAIT_FOR_SIGNAL": "0"},
]
for extra in SETTINGS:
    env = dict(os.environ, **extra)
    print("==", extra or "defaults", flush=True)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "launch_cost.py"), "--quick"], env=env,
                       capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr[-500:] if r.returncode else "", flush=True)
    if r.returncode:
        sys.exit(r.returncode)
