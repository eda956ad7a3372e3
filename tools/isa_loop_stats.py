"""Static instruction counts of a kernel's pass-1 streaming loop (the first loop whose header
issues global loads), per point. Diagnostic for VALU-issue-bound tuning:
    python tools/isa_loop_stats.py [-D...] [--kernel NAME] [--src FILE] [--ppl 16]
Compiles the source for gfx950 (device only) with the given extra defines."""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]


def main(argv):
    defs = [a for a in argv if a.startswith("-D")]
    kern = "_Z15cg_frame_kernelILi128ELi1ELi0ELb0EEv8CgLaunch11CgDevParams"
    src = f"{ROOT}/cones_perception_amd/csrc/cg_kernels.hip"
    ppl = 16
    for i, a in enumerate(argv):
        if a == "--kernel": kern = argv[i + 1]
        if a == "--src": src = argv[i + 1]
        if a == "--ppl": ppl = int(argv[i + 1])
    cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950",
           "-I", f"{ROOT}/include", "--cuda-device-only", "-S", "-o", "/tmp/_isa.s", src,
           "-Rpass-analysis=kernel-resource-usage", *defs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-3000:])
    res = {}
    grab = False
    for l in r.stderr.splitlines():
        if "Function Name:" in l:
            grab = kern in l
        elif grab:
            m = re.search(r"remark:\s+(.*?): (\S+)", l)
            if m: res[m.group(1)] = m.group(2)
    s = open("/tmp/_isa.s").read()
    a = s.index(kern + ":")
    body = s[a: s.index(".Lfunc_end", a)].split("\n")
    hdr = None
    cnt = {"valu": 0, "salu": 0, "vmem": 0, "lds": 0, "writelane": 0, "readlane": 0, "smem": 0, "nop": 0}
    inloop = False
    for l in body:
        t = l.strip()
        m = re.match(r"^(\.LBB\d+_\d+):\s*;\s*=>This Inner Loop Header", t)
        if m and hdr is None:
            # the first loop with global loads in its header region
            hdr = m.group(1)[1:] if m else None
            inloop = True
            continue
        if hdr and re.match(r"^\.LBB\d+_\d+:", t) or (hdr and t.startswith("; %bb.")):
            inloop = f"Header={hdr.replace('LBB', 'BB')}" in t or t.startswith("; %bb.") and inloop
            if re.match(r"^\.LBB\d+_\d+:", t) and f"Header={hdr.replace('LBB', 'BB')}" not in t:
                if cnt["vmem"] == 0:   # not the streaming loop: keep looking
                    hdr = None
                    inloop = False
                    cnt = dict.fromkeys(cnt, 0)
                    continue
                break
            continue
        if not inloop or not t or t.startswith(";") or t.startswith("."):
            continue
        op = t.split()[0]
        if op.startswith("v_writelane"): cnt["writelane"] += 1
        if op.startswith("v_readlane"): cnt["readlane"] += 1
        if op.startswith("v_"): cnt["valu"] += 1
        elif op.startswith("global_") or op.startswith("buffer_"): cnt["vmem"] += 1
        elif op.startswith("ds_"): cnt["lds"] += 1
        elif op.startswith("s_load") or op.startswith("s_buffer"): cnt["smem"] += 1
        elif op.startswith("s_nop"): cnt["nop"] += 1
        elif op.startswith("s_") and not op.startswith("s_waitcnt"): cnt["salu"] += 1
    per = {k: round(v / ppl, 2) for k, v in cnt.items()}
    print({"defines": defs, "VGPRs": res.get("VGPRs"), "SGPRs": res.get("TotalSGPRs"),
           "SGPR spill": res.get("SGPRs Spill"), "per_point": per})


if __name__ == "__main__":
    main(sys.argv[1:])
