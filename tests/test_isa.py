"""Static ISA checks of the built library (no GPU): every gfx950 code object in
libcones_gpu.so is disassembled and must contain no out-of-line call (s_swappc_b64).

Two out-of-line device calls in this code base preceded failures that were never explained
("Lessons"): an exact atan2f called from divergent loops (run-to-run keep-word
changes) and a non-inlined single-wave sort taking a struct through scratch (a GPU memory
fault in a probe). Every device function on the path is force-inlined instead; this test keeps
it that way.

The metadata check goes further: no kernel of the library may use scratch at all (private
segment size 0, no dynamic stack), so no dispatch of ours depends on the runtime provisioning
per-lane scratch. DESIGN.md ("Lessons") records what a rebuilt out-of-line probe shows: a
VGPR value passed by reference lives in the private segment and the callee reaches it with
flat loads through the private aperture.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("CONES_GPU_LIB") or os.path.join(ROOT, "cones_perception_amd", "lib", "libcones_gpu.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _code_objects(tmp_path):
    """The gfx950 code objects of the library's fat binary, one per HIP translation unit."""
    fat = tmp_path / "fat.bin"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", LIB, str(tmp_path / "x.so")],
                   check=True)
    data = fat.read_bytes()
    offs = []
    i = data.find(MAGIC)
    while i >= 0:
        offs.append(i)
        i = data.find(MAGIC, i + 1)
    out = []
    for k, o in enumerate(offs):   # one bundle per translation unit
        b = tmp_path / f"b{k}.bin"
        b.write_bytes(data[o: offs[k + 1] if k + 1 < len(offs) else len(data)])
        co = tmp_path / f"c{k}.co"
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={b}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        out.append(co)
    return out


def _disassembly(tmp_path):
    return [subprocess.run([f"{LLVM}/llvm-objdump", "-d", str(co)], capture_output=True, text=True,
                           check=True).stdout for co in _code_objects(tmp_path)]


def _kernel_metadata(tmp_path):
    """(name, {key: value}) per kernel, from each code object's AMDGPU metadata note."""
    kernels = []
    for co in _code_objects(tmp_path):
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], capture_output=True, text=True,
                               check=True).stdout
        cur = None
        for line in notes.splitlines():
            t = line.strip()
            if t.startswith("- .agpr_count:"):       # first key of each kernel's map
                cur = {}
                kernels.append(cur)
            if cur is not None and t.startswith(".") and ":" in t:
                k, v = t.split(":", 1)
                if v.strip():
                    cur[k.strip()] = v.strip()
            elif cur is not None and t.startswith("- .") and ":" in t:
                k, v = t[2:].split(":", 1)
                cur.setdefault(k.strip(), v.strip())
    return [(k.get(".name"), k) for k in kernels]


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_no_out_of_line_calls_in_device_code(tmp_path):
    units = _disassembly(tmp_path)
    assert len(units) >= 4, "expected one gfx950 code object per HIP source"
    kernels = 0
    for text in units:
        fn = None
        for line in text.splitlines():
            if line.endswith(">:"):
                fn = line
                kernels += 1
            assert "s_swappc_b64" not in line, f"out-of-line call in {fn}: {line.strip()}"
    assert kernels > 50


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_no_kernel_uses_scratch(tmp_path):
    kernels = _kernel_metadata(tmp_path)
    assert len(kernels) > 50
    bad = [(n, m.get(".private_segment_fixed_size"), m.get(".uses_dynamic_stack"), m.get(".vgpr_spill_count"))
           for n, m in kernels
           if m.get(".private_segment_fixed_size") != "0" or m.get(".uses_dynamic_stack") != "false"
           or m.get(".vgpr_spill_count", "0") != "0"]
    assert not bad, f"kernels with scratch (private segment, dynamic stack, VGPR spills): {bad}"


def test_out_of_line_probe_needs_scratch(tmp_path):
    """The mechanism behind the round-2 probe fault, read from a rebuilt probe (tools/
    scratch_probe.hip): a VGPR value passed by reference to an out-of-line device function
    lives in the private segment, which the callee reaches with flat accesses; the stack is
    static (no dynamic stack)."""
    co = tmp_path / "probe.co"
    src = os.path.join(ROOT, "tools", "scratch_probe.hip")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "--no-gpu-bundle-output",
                    "-c", src, "-o", str(co)], check=True, capture_output=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], capture_output=True, text=True,
                           check=True).stdout
    meta = dict(l.strip().split(":", 1) for l in notes.splitlines() if l.strip().startswith((".private_segment", ".uses_dyn")))
    assert int(meta[".private_segment_fixed_size"]) > 0 and meta[".uses_dynamic_stack"].strip() == "false", meta
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", str(co)], capture_output=True, text=True, check=True).stdout
    assert "s_swappc_b64" in dis and "scratch_store_dword" in dis and "flat_load_dword" in dis


def _find(kernels, prefix):
    out = [(n, m) for n, m in kernels if n and n.startswith(prefix)]
    assert out, f"no kernel named {prefix}*"
    return out


def _vgprs(m):   # allocated: gfx950 hands out VGPRs in blocks of 8
    return (int(m[".vgpr_count"]) + 7) // 8 * 8


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_occupancy_contracts(tmp_path):
    """The residency each launch structure is designed around, from the code-object metadata
    (160 KiB of LDS and 512 VGPRs per SIMD lane on a gfx950 CU; a 512-lane workgroup puts two
    waves on each SIMD, a 256-lane one one wave):
      - the fused frame kernel: two workgroups per CU (LDS <= 80 KiB, <= 128 VGPRs).
    And the batch entry point has one launch structure: none of the slower diagnostic batch
    structures of round 3 (front + backend launches, served backends, half-frame pairs, with
    cross-launch waits) is in the library."""
    k = _kernel_metadata(tmp_path)
    lds = lambda m: int(m[".group_segment_fixed_size"])
    frames = _find(k, "_Z15cg_frame_kernelILi128E")
    for n, m in frames:
        assert 2 * lds(m) <= 163840 and 4 * _vgprs(m) <= 512, (n, lds(m), m[".vgpr_count"])
    for gone in ("cg_front_kernel", "cg_back_kernel", "cg_serve_kernel", "cg_pair_kernel", "cg_back_big_kernel",
                 "cg_back_list_kernel"):
        assert not [n for n, _ in k if n and gone in n], gone
