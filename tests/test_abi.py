"""The C-ABI library builds, loads without a GPU, and exports every symbol of include/*.h."""
import os
import re
import subprocess

from conftest import ROOT


def header_symbols():
    """Every function declared by the C headers in include/ (gdf.h, gdf_driver.h)."""
    syms = set()
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if h.endswith(".h"):
            txt = open(os.path.join(ROOT, "include", h)).read()
            syms |= set(re.findall(r"^\s*(?:int|const char\*)\s+(gdf_\w+)\s*\(", txt, re.M))
    return sorted(syms)


def test_library_exports_every_header_symbol():
    from ros_gpu_depthmap_fusion_amd import build_library
    lib = build_library()
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (gdf_\w+)$", out, re.M))
    syms = header_symbols()
    assert len(syms) >= 40
    missing = [s for s in syms if s not in exported]
    assert not missing, missing


def test_python_binding_covers_header():
    from ros_gpu_depthmap_fusion_amd.gdf import EXPORTED
    assert sorted(EXPORTED) == header_symbols()


def test_library_loads_and_reports_version():
    import ctypes
    from ros_gpu_depthmap_fusion_amd.gdf import load_library
    lib = load_library()
    a, b = ctypes.c_int(), ctypes.c_int()
    assert lib.gdf_version(ctypes.byref(a), ctypes.byref(b)) == 0
    assert (a.value, b.value) == (0, 4)
    # null-handle calls fail cleanly with GDF_ERR_ARG, no GPU touched
    assert lib.gdf_clear(None) == -1
    assert b"null engine" in lib.gdf_last_error()


def test_code_object_targets_gfx950():
    from ros_gpu_depthmap_fusion_amd import build_library
    data = open(build_library(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_build_provenance_matches_sources():
    """libgdf.so carries the digest of the sources it was compiled from (gdf_build_info); the
    binding refuses a library built from other sources (no stale build is ever loaded)."""
    from ros_gpu_depthmap_fusion_amd.build import source_digest
    from ros_gpu_depthmap_fusion_amd.gdf import build_info, load_library
    info = build_info(load_library())
    assert info["source_sha"] == source_digest()
    assert info.get("built_on") and info.get("built_at")


def test_local_world_lifecycle_without_gpu():
    """gdf_fused_local_create / _destroy (the in-process transport's world) touch no GPU: argument
    checks, a world of 1..16 ranks, and gdf_fused_info / gdf_fused_create_local refusing nulls."""
    import ctypes
    from ros_gpu_depthmap_fusion_amd.gdf import load_library
    lib = load_library()
    h = ctypes.c_void_p()
    assert lib.gdf_fused_local_create(0, ctypes.byref(h)) == -1
    assert lib.gdf_fused_local_create(17, ctypes.byref(h)) == -1
    assert lib.gdf_fused_local_create(4, ctypes.byref(h)) == 0 and h.value
    out = ctypes.c_void_p()
    assert lib.gdf_fused_create_local(None, h, 0, 4, None, 0, ctypes.byref(out)) == -1
    assert lib.gdf_fused_info(None, None, None, None, None) == -1
    assert lib.gdf_fused_local_destroy(h) == 0
    assert lib.gdf_fused_local_destroy(None) == 0


def kernel_private_segments(lib_path):
    """{kernel symbol: private_segment_fixed_size} of the gfx950 code object inside lib_path
    (llvm-objcopy + clang-offload-bundler + llvm-readelf --notes from /opt/rocm/lib/llvm/bin)."""
    import tempfile
    llvm = "/opt/rocm/lib/llvm/bin"
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "gdf.co")
        subprocess.run([f"{llvm}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", lib_path],
                       check=True, capture_output=True)
        subprocess.run([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}",
                        f"--output={co}"], check=True, capture_output=True)
        notes = subprocess.run([f"{llvm}/llvm-readelf", "--notes", co], check=True,
                               capture_output=True, text=True).stdout
    names = re.findall(r"^\s+\.name:\s+(\S+)\s*$", notes, re.M)
    sizes = [int(x) for x in re.findall(r"\.private_segment_fixed_size:\s+(\d+)", notes)]
    assert len(names) == len(sizes) > 20
    return dict(zip(names, sizes))


def test_no_kernel_keeps_a_private_copy_of_its_arguments():
    """Round 4's k_mask_px_o8 fault: the compiler kept a private (scratch) copy of the 2 KB
    by-value FrameArgs, and the kernels' global loads of the camera table then addressed scratch
    (HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION).  cam_table() now addresses the kernarg segment
    itself; this pins the consequence: no kernel of the library spends more than 256 B of scratch
    per lane (a copy of FrameArgs is > 2 KB; register spills of the frame kernels are <= 48 B)."""
    from ros_gpu_depthmap_fusion_amd import build_library
    sizes = kernel_private_segments(build_library())
    frame = {k: v for k, v in sizes.items() if "FrameArgs" in k}
    assert len(frame) >= 6
    big = {k: v for k, v in sizes.items() if v > 256}
    assert not big, big
