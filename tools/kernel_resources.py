"""Per-kernel register / scratch / occupancy report of one HIP source (hipcc
-Rpass-analysis=kernel-resource-usage, device-only compile for gfx950): spills show up as a
non-zero ScratchSize.  python tools/kernel_resources.py csrc/kernels/flash_attn.hip [name-filter]"""
import os
import re
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "csrc"))


def main():
    import build
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    inc, _, abi = build._torch_paths()
    flags = ["-O3", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_API_INCLUDE_EXTENSION_H",
             "-I" + os.path.join(ROOT, "csrc", "include"), "-I" + sysconfig.get_paths()["include"]]
    flags += ["-I" + p for p in inc]
    flags += [f"--offload-arch={build.ARCH}", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-fno-gpu-rdc",
              "-munsafe-fp-atomics", "-Wno-unused-result", "-Wno-return-type", "-ffp-contract=fast",
              "--offload-device-only", "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(["hipcc"] + flags + ["-c", src, "-o", "/tmp/_kres.o"], capture_output=True, text=True)
    cur, rows = None, []
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+([A-Za-z][A-Za-z /\[\]]*?): (.*?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    if r.returncode != 0:
        print(r.stderr[-3000:])
    for d in rows:
        if filt in d["name"]:
            print(f"{d['name'][:70]:70s} VGPR {d.get('VGPRs', '?'):>4} AGPR {d.get('AGPRs', '?'):>4} "
                  f"spill {d.get('VGPRs Spill', '?'):>4} scratch {d.get('ScratchSize [bytes/lane]', '?'):>4} "
                  f"occ {d.get('Occupancy [waves/SIMD]', '?')}")


if __name__ == "__main__":
    main()
