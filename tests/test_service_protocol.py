"""The decode service's wire protocol (include/sdsj.h sdsj_svc_req / sdsj_svc_rep) and the worker-side
client (sds_amd/service.py), on the CPU: a stand-in server written here from the header's description
(map the client's memfd, read the input at [0, in_len), write the output at out_off, reply {seq,
status}) exercises the client's region growth, ordering and frame requests.  The native loop itself
(sds_amd/csrc/sdsj_service.hip) runs under -m gpu (tests/test_gpu_dropin.py service cases)."""
import mmap
import os
import re
import socket
import threading
import uuid

import numpy as np
import pytest

from sds_amd import _lib
from sds_amd import service as S

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_struct_layout_matches_the_header():
    text = open(os.path.join(REPO, "include", "sdsj.h")).read()
    assert "} sdsj_svc_req; /* 72 bytes */" in text and "} sdsj_svc_rep; /* 16 bytes */" in text
    assert S._REQ.size == 72 and S._REP.size == 16
    assert int(re.search(r"#define SDSJ_SVC_MAGIC (0x[0-9A-Fa-f]+)u", text).group(1), 16) == S.MAGIC
    for name, v in (("MAP", S.KIND_MAP), ("DECODE", S.KIND_DECODE), ("FRAME", S.KIND_FRAME)):
        assert f"#define SDSJ_SVC_{name} {v}" in text


class _StandIn(threading.Thread):
    """Stand-in service: DECODE writes out_bytes(op) bytes of value (sum of input bytes + flip) % 256;
    FRAME writes the frame's first output-size bytes; a request beyond the region replies EINVAL."""

    def __init__(self, address):
        super().__init__(daemon=True)
        self.lsock = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
        self.lsock.bind(b"\0" + address.encode())
        self.lsock.listen(8)
        self.maps = 0

    def run(self):
        conn, _ = self.lsock.accept()
        mm = None
        while True:
            try:
                msg, fds, _, _ = socket.recv_fds(conn, S._REQ.size, 1)
            except OSError:
                return
            if not msg:
                return
            f = S._REQ.unpack(msg)
            magic, kind, seq, in_len, out_off, w, h = f[:7]
            out_h, out_w, _crop, _filt, dtype, _lay, flip = f[7:14]
            st = 0
            if kind == S.KIND_MAP:
                if mm is not None:
                    mm.close()
                mm = mmap.mmap(fds[0], in_len)
                os.close(fds[0])
                self.maps += 1
            else:
                ob = out_h * out_w * 3 * (4 if dtype == 1 else 1)
                if out_off + ob > len(mm) or in_len > len(mm):
                    st = -1
                elif kind == S.KIND_DECODE:
                    v = (sum(mm[0:in_len]) + flip) % 256
                    mm[out_off:out_off + ob] = bytes([v]) * ob
                else:
                    src = np.frombuffer(mm[0:w * h * 3], np.uint8)
                    mm[out_off:out_off + ob] = np.resize(src, ob).tobytes()
            conn.send(S._REP.pack(seq, st, 0))


def test_client_against_a_stand_in_service():
    addr = f"sds_amd-test-{uuid.uuid4().hex[:8]}"
    srv = _StandIn(addr)
    srv.start()
    c = S.ServiceClient(addr)
    op = _lib.SdsjOp(16, 8, 1, 1, _lib.DTYPE_U8, _lib.LAYOUT_HWC)
    rng = np.random.default_rng(0)
    for n in (10, 1000, 9 << 20, 100):  # the 9 MiB sample grows the region (a second MAP)
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for flip in (False, True):
            st, arr = c.decode(data, op, flip)
            assert st == 0 and arr.shape == (16, 8, 3) and arr.dtype == np.uint8
            assert (arr == (sum(data) + flip) % 256).all()
    assert srv.maps == 2 and c.size >= 9 << 20
    opf = _lib.SdsjOp(4, 5, 1, 1, _lib.DTYPE_F32, _lib.LAYOUT_CHW)
    st, arr = c.decode(b"\x01\x02", opf)
    assert st == 0 and arr.shape == (3, 4, 5) and arr.dtype == np.float32
    frame = rng.integers(0, 256, (7, 9, 3), dtype=np.uint8)
    st, arr = c.resize_frame(frame, op)
    assert st == 0 and np.array_equal(arr.reshape(-1), np.resize(frame.reshape(-1), 16 * 8 * 3))
    big = _lib.SdsjOp(4096, 4096, 1, 1, _lib.DTYPE_F32, _lib.LAYOUT_HWC)  # 201 MB output: region grows again
    st, arr = c.decode(b"\x00", big)
    assert st == 0 and srv.maps == 3
    c.close()


def test_pipeline_starts_no_service_without_a_gpu():
    import torch
    if torch.cuda.device_count():
        pytest.skip("GPU present")
    from sds_amd.presets import create_standard_image_pipeline
    ts = create_standard_image_pipeline("jpg", (256, 256))
    assert ts[1].service_address is None and not S._handles


def test_service_process_lifecycle_without_a_gpu():
    """The launcher (sds_amd.service.ensure_service): the service process binds its address before
    initialising anything (a client can connect at once), exits on SIGTERM while idle, and -- once a
    client connects -- initialises HIP in its own process; without a GPU the native loop reports the
    error and the process exits non-zero instead of hanging."""
    import time
    import torch
    if torch.cuda.device_count():
        pytest.skip("GPU present")
    addr = S.ensure_service(0)
    h = S._handles[(os.getpid(), 0)]
    assert S.ensure_service(0) == addr  # one service per (process, device)
    deadline = time.time() + 60
    sock = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    while True:
        try:
            sock.connect(b"\0" + addr.encode())
            break
        except (ConnectionRefusedError, FileNotFoundError):
            assert time.time() < deadline, "service never listened"
            time.sleep(0.05)
    assert h.proc.wait(timeout=120) != 0  # no GPU: sdsj_service_serve fails, the process exits
    sock.close()
    del S._handles[(os.getpid(), 0)]
    h2 = S._Handle(0, 1, 8)  # idle (no client): SIGTERM ends it
    time.sleep(0.5)
    h2.stop()
    assert h2.proc.returncode is not None
