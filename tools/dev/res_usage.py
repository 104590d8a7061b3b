"""Per-kernel VGPR / spill / occupancy table of one HIP source (hipcc -Rpass-analysis remarks).
usage: python tools/res_usage.py graph-physics_amd/csrc/mgn_chain16.hip [extra hipcc flags...]"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-mllvm",
       "-amdgpu-mfma-vgpr-form", "-I", "include", "-c", src, "-o", "/tmp/res_usage.o",
       "-Rpass-analysis=kernel-resource-usage", *sys.argv[2:]]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s*(Function Name|VGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    print(f"{r.get('VGPRs','?'):>4} spill {r.get('VGPRs Spill','?'):>3} occ {r.get('Occupancy [waves/SIMD]','?')}  {r['name'][:110]}")
