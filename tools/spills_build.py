"""Registers / spills / scratch of every optimiser kernel as the library is built: compiles each
compilation unit of build.units() with its own flags to device assembly (hipcc -S) and reads the
kernel metadata (tools/spills.py).

    python tools/spills_build.py [out.txt] [-j 8]
"""
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.getcwd())
from irm_motion_planning_amd import build  # noqa: E402

out = next((a for a in sys.argv[1:] if not a.startswith("-") and not a.isdigit()), None)
jobs = int(sys.argv[sys.argv.index("-j") + 1]) if "-j" in sys.argv else 8
tmp = tempfile.mkdtemp()
units = [u for u in build.units() if u[1] == "irm_opt_inst.hip"]


def one(u):
    name, src, flags = u
    s = os.path.join(tmp, name + ".s")
    subprocess.check_call([build.HIPCC] + build.CFLAGS + flags + ["--cuda-device-only", "-S", "-o", s, src],
                          cwd=build.CSRC, stderr=subprocess.DEVNULL)
    r = subprocess.run([sys.executable, "tools/spills.py", s, "k_"], capture_output=True, text=True).stdout
    return name, r


lines = []
with ThreadPoolExecutor(jobs) as ex:
    for name, r in ex.map(one, units):
        lines.append(f"== unit {name}\n{r}")
text = "".join(lines)
print(text)
if out:
    open(out, "w").write(text)
