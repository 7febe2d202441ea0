"""CPU: the C read callback shown in INTEGRATION.md compiles against the reference's own headers
(sr-main.h, sr-types.h) and include/sr_router.h, and links against libsr_router.so: the document's
binding is code, not prose. Skipped where /root/reference is absent (the GPU box)."""
from __future__ import annotations

import os
import re
import subprocess

import pytest

from conftest import REPO

REF = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference headers absent")
def test_integration_callback_compiles(tmp_path):
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    blocks = re.findall(r"```c\n(.*?)```", doc, flags=re.S)
    assert blocks, "no C block in INTEGRATION.md"
    src = tmp_path / "cb.c"
    src.write_text(blocks[0] + "\nint main(void) { void (*cb)(struct ev_loop *, struct ev_io *, int) = udp_read_cb_gpu; return cb == 0; }\n")
    lib = os.path.join(REPO, "statsd-router_amd", "lib")
    p = subprocess.run(["gcc", "-Wall", "-Werror", "-Wno-unused-function", "-Wno-strict-aliasing", "-fcommon",
                        "-I", REF, "-I", os.path.join(REPO, "include"), "-I", "/opt/conda/include", str(src),
                        "-o", str(tmp_path / "cb"), "-L", lib, "-lsr_router", "-lsr_route",
                        "-Wl,-rpath-link,/usr/lib/x86_64-linux-gnu", "/opt/conda/lib/libev.so.4",
                        os.path.join(REF, "sr-util.c")],
                       capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
