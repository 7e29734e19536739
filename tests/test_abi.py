"""The C-ABI library: builds, loads, exports every entry point include/raytracer_hip.h
declares, host-only helpers (camera math) match the oracle, and -- with no GPU in this
container -- context creation fails loudly instead of falling back to the CPU."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from raytracer_hip import abi, scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "raytracer_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(rt_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_expected_api():
    names = declared_functions()
    assert len(names) == len(abi.EXPORTS), names
    assert set(names) == {n for n, _, _ in abi.EXPORTS}


def test_csharp_shim_binds_declared_entry_points_and_checks_the_abi():
    """shim/csharp/RayTracer.cs: every [DllImport] is an entry point the header declares, and the constructor
    compares rt_abi_version() with the ABI the binding was written for (RT_ABI_VERSION) before anything else."""
    src = open(os.path.join(ROOT, "shim", "csharp", "RayTracer.cs")).read()
    externs = re.findall(r"\[DllImport\(Lib\)\]\s+internal static extern \w+ (rt_\w+)\(", src)
    assert externs and set(externs) <= set(declared_functions()), set(externs) - set(declared_functions())
    assert "rt_abi_version" in externs
    want = int(re.search(r"#define RT_ABI_VERSION (\d+)", open(HEADER).read()).group(1))
    assert int(re.search(r"internal const int AbiVersion = (\d+);", src).group(1)) == want == abi.RT_ABI_VERSION
    ctor = src[src.index("public RayTracer(Surface screen)"):]
    assert ctor.index("rt_abi_version()") < ctor.index("rt_create(")


def test_library_exports_every_declared_symbol(rtlib):
    out = subprocess.run(["nm", "-D", "--defined-only", abi.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    for n in declared_functions():
        assert getattr(rtlib, n) is not None


def test_library_is_gfx950_code_object(rtlib):
    """The .so embeds a gfx950 code object (hipcc --offload-arch=gfx950) and nothing else."""
    blob = open(abi.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"gfx942" not in blob and b"sm_" + b"90" not in blob


def test_struct_layouts_match_header():
    assert C.sizeof(abi.rt_vec3) == 12
    assert C.sizeof(abi.rt_material) == 52   # C# Material is 52 B as well (RayTracer.cs:60-80)
    assert C.sizeof(abi.rt_sphere) == 68
    assert C.sizeof(abi.rt_plane) == 76
    assert C.sizeof(abi.rt_light) == 16
    assert C.sizeof(abi.rt_camera) == 20
    assert C.sizeof(abi.rt_stats) == 8 * 8 + 4 * 8 + 3 * 8
    assert C.sizeof(abi.rt_work) == 8 * 8


def test_abi_version(rtlib):
    # 10: rt_set_counting (9: the per-worker Tick hand-off, RT_CREATE_SHARED_DEVICE; 8: rt_comm_probe; 7: rt_comm_*)
    assert rtlib.rt_abi_version() == 10 == abi.RT_ABI_VERSION
    hdr = open(HEADER).read()
    assert re.search(r"#define RT_ABI_VERSION (\d+)", hdr).group(1) == str(abi.RT_ABI_VERSION)
    assert re.search(r"RT_CREATE_RCCL_GATHER = (\d+), RT_CREATE_SHARED_DEVICE = (\d+)", hdr).groups() == \
        (str(abi.RT_CREATE_RCCL_GATHER), str(abi.RT_CREATE_SHARED_DEVICE))
    assert re.search(r"#define RT_MAX_WORKERS (\d+)", hdr).group(1) == str(abi.RT_MAX_WORKERS)


def test_create_flag_checks(rtlib):
    """rt_create_ex's argument checks come before any device query (they hold on a CPU-only host): unknown
    flags, n_gpus outside [1, RT_MAX_WORKERS], and RCCL_GATHER with SHARED_DEVICE at n > 1 (RCCL refuses two
    ranks on one device) are argument errors."""
    out = C.c_void_p()
    for n, flags in [(1, 4), (0, 0), (abi.RT_MAX_WORKERS + 1, abi.RT_CREATE_SHARED_DEVICE),
                     (2, abi.RT_CREATE_RCCL_GATHER | abi.RT_CREATE_SHARED_DEVICE)]:
        assert rtlib.rt_create_ex(n, flags, C.byref(out)) == abi.RT_ERR_INVALID_ARG, (n, flags)
        assert not out.value


def test_camera_view_matches_oracle(rtlib, oracle):
    ol = oracle.lib()
    for cam in [abi.rt_camera(abi.rt_vec3(0, 0, 0), 0.0, 0.0),
                abi.rt_camera(abi.rt_vec3(1.5, -0.25, 3.0), 0.7, -0.3),
                abi.rt_camera(abi.rt_vec3(0, 0, 0), -2.9, 1.4)]:
        for (w, h) in [(512, 512), (1920, 1080), (7, 3)]:
            a, b = abi.rt_view(), abi.rt_view()
            assert rtlib.rt_camera_view(C.byref(cam), w, h, C.byref(a)) == 0
            assert ol.oracle_camera_view(C.byref(cam), w, h, C.byref(b)) == 0
            assert bytes(a) == bytes(b)


def _basis(cam):
    """CameraForward/Right/Up restated in numpy (RayTracer.cs:511-523)."""
    import math
    f32 = np.float32
    p, y = float(cam.pitch), float(cam.yaw)
    F = np.array([math.cos(p) * math.sin(y), -math.sin(p), math.cos(p) * math.cos(y)]).astype(f32)
    R = np.array([math.cos(y), 0.0, -math.sin(y)]).astype(f32)
    U = np.array([R[1] * F[2] - R[2] * F[1], R[2] * F[0] - R[0] * F[2], R[0] * F[1] - R[1] * F[0]], dtype=f32)
    return F, R, U


def test_on_key_press_semantics(rtlib):
    """OnKeyPress, RayTracer.cs:543-554: W/S along forward, A/D along right, Space/Shift along up."""
    f32 = np.float32
    cam = abi.rt_camera(abi.rt_vec3(0.5, 0.25, -1.0), 0.4, -0.2)
    for key, which, sign in [(abi.RT_KEY_W, 0, 1), (abi.RT_KEY_S, 0, -1), (abi.RT_KEY_A, 1, -1),
                             (abi.RT_KEY_D, 1, 1), (abi.RT_KEY_SPACE, 2, -1), (abi.RT_KEY_SHIFT, 2, 1)]:
        c = abi.rt_camera.from_buffer_copy(cam)
        pos = np.array(c.position.tuple(), dtype=f32)
        d = _basis(c)[which] * f32(0.05)
        want = pos + d if sign > 0 else pos - d
        assert rtlib.rt_camera_on_key(C.byref(c), key) == 0
        assert np.array_equal(np.array(c.position.tuple(), dtype=f32), want)
    c = abi.rt_camera.from_buffer_copy(cam)
    assert rtlib.rt_camera_on_key(C.byref(c), 99) == 0 and bytes(c) == bytes(cam)  # `_ => _cameraPosition`


def test_on_mouse_move_semantics(rtlib):
    f32 = np.float32
    c = abi.rt_camera(abi.rt_vec3(0, 0, 0), 0.1, -0.2)
    assert rtlib.rt_camera_on_mouse_move(C.byref(c), 7.0, -3.5) == 0
    assert c.yaw == float(f32(0.1) + f32(7.0) / f32(360))
    assert c.pitch == float(f32(-0.2) + f32(-3.5) / f32(360))


def test_null_arguments_are_errors(rtlib):
    assert rtlib.rt_camera_view(None, 4, 4, None) == abi.RT_ERR_INVALID_ARG
    assert rtlib.rt_last_error(None)
    assert rtlib.rt_set_scene(None, None, 0, None, 0, None, 0, abi.rt_vec3(0, 0, 0), 0) == abi.RT_ERR_INVALID_ARG
    assert rtlib.rt_render(None, 4, 4, None) == abi.RT_ERR_INVALID_ARG
    assert rtlib.rt_create(0, C.byref(C.c_void_p())) == abi.RT_ERR_INVALID_ARG
    assert rtlib.rt_create_ex(1, 0x100, C.byref(C.c_void_p())) == abi.RT_ERR_INVALID_ARG  # unknown flag
    assert rtlib.rt_count_work(None, 4, 4, None) == abi.RT_ERR_INVALID_ARG
    assert rtlib.rt_set_timing(None, 1) == abi.RT_ERR_INVALID_ARG
    assert rtlib.rt_dispatch_order(None, C.byref(C.c_int())) == abi.RT_ERR_INVALID_ARG
    assert rtlib.rt_debug_segments(None, 4, 4, 1, None, 0, C.byref(C.c_int())) == abi.RT_ERR_INVALID_ARG


def test_no_cpu_fallback_without_gpu(rtlib):
    """In this GPU-less container rt_create must fail with RT_ERR_NO_DEVICE, not render on the CPU."""
    n = C.c_int(-1)
    assert rtlib.rt_device_count(C.byref(n)) == 0
    if n.value > 0:
        pytest.skip("a GPU is visible")
    p = C.c_void_p()
    assert rtlib.rt_create(1, C.byref(p)) == abi.RT_ERR_NO_DEVICE
    assert b"no HIP device" in rtlib.rt_last_error(None)
    from raytracer_hip import RayTracer, RayTracerError, Surface
    with pytest.raises(RayTracerError):
        RayTracer(Surface(8, 8))


def test_scene_generator_deterministic():
    a = scenes.config("C4")
    b = scenes.config("C4")
    assert a.spheres == b.spheres and len(a.spheres) == 64 and len(a.planes) == 2 and len(a.lights) == 4
    c2 = scenes.config("C2")
    assert c2.spheres == a.spheres[:8]
    assert scenes.config("C3").recursion_limit == 3 and scenes.config("C5").width == 7680
    for s in a.spheres[3:]:
        for v in s.center + (s.radius,):
            assert v * 64 == int(v * 64)  # quantised to 1/64
    # SplitMix64 known answers (seed 0): the generator is the published algorithm
    sm = scenes.SplitMix64(0)
    assert sm.next() == 0xE220A8397B1DCDAF
    assert sm.next() == 0x6E789E6AA1B965F4


def test_reference_scene_verbatim():
    sc = scenes.reference()
    assert sc.recursion_limit == 32
    assert sc.ambient[0] == float(np.float32(43) / np.float32(255))
    red, green, mirror = sc.spheres
    assert red.center == (2.5, 0.0, 8.0) and red.material.kd == (1.0, 0.0, 0.0) and red.material.ks == (0, 0, 0)
    assert green.material.ks == (float(np.float32(0.4)),) * 3 and green.material.n == 1.0
    assert mirror.material.km == (1.0, 1.0, 1.0) and mirror.material.kd == (0, 0, 0)
    pl = sc.planes[0]
    assert pl.material.n == 0.5 and pl.material.km == (1.0, 1.0, 1.0) and pl.material.ka == (0.5, 0.5, 0.5)


def test_write_ppm_roundtrip(tmp_path):
    """Headless display hand-off (rt_write_ppm): P6 header and RGB bytes from 0x00RRGGBB."""
    from raytracer_hip import Surface
    s = Surface(5, 3)
    s.pixels[:] = np.arange(15, dtype=np.int32) * 0x010203 + 0x00102030
    path = str(tmp_path / "f.ppm")
    s.save_ppm(path)
    data = open(path, "rb").read()
    head = b"P6\n5 3\n255\n"
    assert data.startswith(head)
    rgb = np.frombuffer(data[len(head):], dtype=np.uint8).reshape(15, 3)
    u = s.pixels.view(np.uint32)
    assert (rgb[:, 0] == (u >> 16) & 255).all() and (rgb[:, 1] == (u >> 8) & 255).all() and (rgb[:, 2] == u & 255).all()
    lib = abi.load_library()
    assert lib.rt_write_ppm(None, None, 1, 1) == abi.RT_ERR_INVALID_ARG


def test_ctypes_layouts_match_the_c_header(tmp_path):
    """sizeof/offsetof of every ABI struct, from gcc on include/raytracer_hip.h, against the
    ctypes mirror (what the C#/Go/Python bindings must reproduce)."""
    import subprocess
    structs = {n: getattr(abi, n) for n in ("rt_vec3", "rt_material", "rt_sphere", "rt_plane", "rt_light",
                                           "rt_camera", "rt_view", "rt_segment", "rt_stats", "rt_work", "rt_wire_layout")}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "raytracer_hip.h"', "int main(void) {"]
    for n, t in structs.items():
        lines.append(f'printf("{n} %zu\\n", sizeof({n}));')
        for f, _ in t._fields_:
            lines.append(f'printf("{n}.{f} %zu\\n", offsetof({n}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                  check=True).stdout.splitlines())
    for n, t in structs.items():
        assert int(got[n]) == C.sizeof(t), n
        for f, _ in t._fields_:
            assert int(got[f"{n}.{f}"]) == getattr(t, f).offset, f"{n}.{f}"


def test_bit_pattern_selection_rule():
    """rt_kernel.hip take_primary / take_secondary select on bit patterns: with u(x) = bits(x) - 1
    (uint32, wrapping), `x > 0 && x < best` == `u(x) < u(best)` whenever best is +inf or a positive
    float (the only values a nearest-hit search holds).  Checked on every special value and on
    random bit patterns against the IEEE comparison."""
    rng = np.random.default_rng(7)
    special = np.array([0x00000000, 0x80000000, 0x00000001, 0x80000001, 0x007fffff, 0x00800000, 0x3f800000,
                        0xbf800000, 0x7f7fffff, 0xff7fffff, 0x7f800000, 0xff800000, 0x7f800001, 0x7fc00000,
                        0x7fffffff, 0xff800001, 0xffc00000, 0xffffffff], dtype=np.uint32)
    xs = np.concatenate([special, rng.integers(0, 2**32, 200_000, dtype=np.uint64).astype(np.uint32)])
    pos = xs[(xs.view(np.float32) > 0) & np.isfinite(xs.view(np.float32))]
    bests = np.concatenate([np.array([0x7f800000], dtype=np.uint32), special[[2, 4, 5, 6, 8]], pos[:300]])
    u = lambda b: (b.astype(np.uint64) - 1) % 2**32  # noqa: E731
    with np.errstate(invalid="ignore"):
        for b in bests:
            bf = np.array([b], dtype=np.uint32).view(np.float32)[0]
            ref = (xs.view(np.float32) > 0) & (xs.view(np.float32) < bf)
            assert np.array_equal(ref, u(xs) < u(np.array([b], dtype=np.uint32))[0]), hex(int(b))
