"""r05/r06: which sequence leaves the process aborting at exit (glibc "double free or corruption" after the Tick
tests, r05b).  One sequence per process:  python tools/probes/exit_abort_probe.py A|B|...|I
RAYTRACER_HIP_LIB selects the library build (tools/probes/exit_abort.sh runs the product build and the two
pre-fix variants, tools/probes/rtld_global.patch and pitched_pageable.patch, over every sequence)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))
import numpy as np  # noqa: E402

from raytracer_hip import Context, abi, scenes  # noqa: E402

sc = scenes.config("C3")
W, H = sc.width, sc.height


def rccl():
    with Context(1, abi.RT_CREATE_RCCL_GATHER) as c:
        c.set_scene(sc)
        c.render(W, H)


def plain(n=1, flags=0, register=True):
    with Context(n, flags) as c:
        c.set_scene(sc)
        px = np.zeros(W * H, dtype=np.int32)
        if register:
            c.register_host(px)
        c.render(W, H, px)
        if register:
            c.unregister_host(px)


seq = {"A": [rccl, plain], "B": [rccl, lambda: plain(2, abi.RT_CREATE_SHARED_DEVICE)],
       "C": [rccl, lambda: plain(1, 0, False)], "D": [lambda: plain(2, abi.RT_CREATE_SHARED_DEVICE), rccl],
       "E": [rccl, rccl], "F": [rccl], "G": [rccl, lambda: __import__("torch").zeros(1, device="cuda").sum().item()],
       # H: an unregistered frame of a 3-worker shared-device Tick (one runtime copy per band; the pitched 2-D
       # copy into pageable memory in the pitched_pageable build); I: torch imported after RCCL, no GPU op
       "H": [lambda: plain(3, abi.RT_CREATE_SHARED_DEVICE, False)],
       "I": [rccl, lambda: __import__("torch")],
       }[sys.argv[1]]
for f in seq:
    f()
print("sequence", sys.argv[1], "done", flush=True)
