"""VGPRs, AGPRs, scratch bytes per lane and waves per SIMD of the data-path kernels (1200-B rows, VEC 16):
hipcc -Rpass-analysis=kernel-resource-usage on fec_engine.hip (profiles/r0N_kernel_resources.txt).
Extra arguments are passed to hipcc (e.g. -DFEC_... variants)."""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c",
       f"{ROOT}/pquic_amd/csrc/fec_engine.hip", "-o", "/dev/null", f"-I{ROOT}/include", f"-I{ROOT}/pquic_amd/csrc",
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
want = re.compile(r"k_rlc_(encode_bs2?|recover_bs2?|encode_rows|encode_sp)<(\d+), (\d+|true|false)>")
rec, cur = {}, None
for ln in out.splitlines():
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        cur = m.group(1)
        rec[cur] = {}
        continue
    for key, pat in (("V", r"VGPRs: (\d+)"), ("A", r"AGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, ln)
        if m and cur:
            rec[cur][key] = int(m.group(1))
rows = []
for name, v in rec.items():
    dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    if want.search(dm):
        rows.append(f"{dm.split('(')[0]:<45} V{v.get('V')} A{v.get('A', 0)} scratch{v.get('scratch')} occ{v.get('occ')}")
print("\n".join(sorted(rows)))
