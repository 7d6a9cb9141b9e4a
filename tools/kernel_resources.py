"""Print per-kernel VGPR/SGPR/spill/LDS/occupancy from hipcc -Rpass-analysis=kernel-resource-usage."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "bikg_graph_explainability_public_amd/csrc/xpgnn.hip"
out = subprocess.run(["hipcc", "--offload-arch=gfx950", "--cuda-device-only", "-O3", "-std=c++17", "-fno-slp-vectorize", "-c", "-o", "/tmp/_kr.o",
                      __import__("os").path.abspath(src), "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True,
                     cwd="/tmp").stderr
cur, rows = None, {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark: +([A-Za-z][A-Za-z \[\]/]*?): (\S+) \[-Rpass", line)
    if cur and m:
        rows[cur][m.group(1).strip()] = m.group(2)
filt = sys.argv[2] if len(sys.argv) > 2 else ""
for name, d in rows.items():
    if filt in name:
        dn = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        dn = re.sub(r"\(anonymous namespace\)::", "", dn).replace("void ", "")
        dn = dn.split("(")[0]
        print(f"{dn[:80]:80s} vgpr={d.get('VGPRs','?'):>4} agpr={d.get('AGPRs','?'):>3} "
              f"sgpr={d.get('SGPRs','?'):>3} vspill={d.get('VGPRs Spill','?')} "
              f"lds={d.get('LDS Size [bytes/block]','?')} occ={d.get('Occupancy [waves/SIMD]','?')}")
