"""Print per-kernel register / LDS / occupancy from hipcc -Rpass-analysis=kernel-resource-usage."""
import re, subprocess, sys
src = sys.argv[1]
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", "include", "-mllvm", "-amdgpu-mfma-vgpr-form", "-c", src,
                      "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None; rows = []
for line in out.splitlines():
    m = re.search(r"remark: (.*)", line)
    if not m: continue
    t = m.group(1).replace(" [-Rpass-analysis=kernel-resource-usage]", "")
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}; rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1); cur[k.strip()] = v.strip()
for r in rows:
    dm = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
    dm = re.sub(r"\(anonymous namespace\)::", "", dm)[:90]
    print(f"{r.get('VGPRs'):>4} v {r.get('AGPRs'):>4} a  scr {r.get('ScratchSize [bytes/lane]'):>3}  occ {r.get('Occupancy [waves/SIMD]'):>2}  lds {r.get('LDS Size [bytes/block]'):>6}  {dm}")
