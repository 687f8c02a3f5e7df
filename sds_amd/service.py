"""Node-local decode service: one GPU-owning process per device, serving the per-sample transforms of
every DataLoader worker (include/sdsj.h sdsj_service_serve; the loop itself is native,
sds_amd/csrc/sdsj_service.hip).

Why: sds runs its transform list per sample inside DataLoader workers forked from the training process
(sds/dataset.py:535-561; examples/iter_image_dataset.py:72-80 uses fork, num_workers=2 and
pin_memory=True, whose parent queries the GPU before forking).  Such a worker cannot initialise HIP, and
one image per call leaves the GPU idle.  The service is started by the process that builds the pipeline
(``create_standard_image_pipeline(..., device='cuda')``), so it exists before any worker forks; a worker's
transform sends its sample's encoded bytes through a shared-memory region and one SOCK_SEQPACKET packet,
the service coalesces the concurrent requests of all workers into batched engine calls, and the worker
gets back a host tensor -- the reference's own output type, so ``pin_memory=True`` pins it.

The service process binds its socket at once and initialises the GPU only when the first worker
connects: a pipeline that is never used from a worker costs one sleeping process.  It exits with its
parent (and on SIGTERM, which the parent sends at exit).
"""
from __future__ import annotations

import atexit
import ctypes
import mmap
import os
import select
import socket
import struct
import subprocess
import sys
import threading
import time
import uuid
from typing import Optional

import numpy as np

# include/sdsj.h sdsj_svc_req / sdsj_svc_rep (little-endian, fixed size)
MAGIC = 0x4A534453
KIND_MAP, KIND_DECODE, KIND_FRAME = 1, 2, 3
_REQ = struct.Struct("<IIQqqii6iii")
_REP = struct.Struct("<Qii")
assert _REQ.size == 72 and _REP.size == 16
OK, EINVAL = 0, -1
CONNECT_TIMEOUT_S = float(os.environ.get("SDS_AMD_SERVICE_TIMEOUT", "300"))
# SDS_AMD_SERVICE_PROFILE=<path>: each worker appends its cumulative per-phase times (seconds) to <path>
# every 256 requests (copy-in, the request's round trip, copy-out) -- tools/persample_bench.py
PROFILE_PATH = os.environ.get("SDS_AMD_SERVICE_PROFILE")


class ServiceError(RuntimeError):
    pass


# ------------------------------------------------------------------------------------------------
# parent side: one service process per (owner process, device)
# ------------------------------------------------------------------------------------------------
class _Handle:
    def __init__(self, device: int, engines: int, max_batch: int):
        self.address = f"sds_amd-{os.getpid()}-{device}-{uuid.uuid4().hex[:12]}"
        self.owner = os.getpid()
        self.device = device
        cmd = [sys.executable, "-m", "sds_amd.service", "--address", self.address, "--device", str(device),
               "--parent", str(os.getpid()), "--engines", str(engines), "--max-batch", str(max_batch)]
        env = dict(os.environ)
        repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env["PYTHONPATH"] = repo + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        # one stream per engine, and one hardware queue per stream (HIP's default is 4 per process)
        if engines > int(env.get("GPU_MAX_HW_QUEUES", "4") or 4):
            env["GPU_MAX_HW_QUEUES"] = str(min(engines, 16))
        self.proc = subprocess.Popen(cmd, stdin=subprocess.DEVNULL, close_fds=True, env=env)
        atexit.register(self.stop)

    def stop(self) -> None:
        if os.getpid() != self.owner or self.proc.poll() is not None:
            return
        self.proc.terminate()
        try:
            self.proc.wait(timeout=20)
        except subprocess.TimeoutExpired:
            self.proc.kill()
            self.proc.wait(timeout=20)


_handles: dict[tuple[int, int], _Handle] = {}
_handles_lock = threading.Lock()


def ensure_service(device: int = 0, engines: int | None = None, max_batch: int = 64) -> str:
    """Starts (once per process and device) the decode service for HIP device ``device``; returns its
    address (an abstract AF_UNIX name).  Call it before DataLoader workers fork -- the pipeline factory
    does.  The process starting it needs no GPU; the service initialises HIP in its own process."""
    if engines is None:
        # 4: the loader-shape sweep (profiles/r05_persample.jsonl) put 4 engines level with 8 at 8 workers
        # and ahead at 16, with a third less service CPU than 8
        engines = int(os.environ.get("SDS_AMD_SERVICE_ENGINES", "4"))
    key = (os.getpid(), int(device))
    with _handles_lock:
        h = _handles.get(key)
        if h is None or h.proc.poll() is not None:
            h = _Handle(int(device), int(engines), int(max_batch))
            _handles[key] = h
        return h.address


# ------------------------------------------------------------------------------------------------
# worker side: one connection and one shared region per (process, address)
# ------------------------------------------------------------------------------------------------
def _align(v: int, a: int = 4096) -> int:
    return (v + a - 1) // a * a


class ServiceClient:
    """The worker's end: its region (a memfd shared with the service) and its connection."""

    def __init__(self, address: str):
        self.address = address
        self.pid = os.getpid()
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
        deadline = time.monotonic() + CONNECT_TIMEOUT_S
        while True:
            try:
                self.sock.connect(b"\0" + address.encode())
                break
            except (ConnectionRefusedError, FileNotFoundError):
                if time.monotonic() > deadline:
                    raise ServiceError(f"decode service {address!r} is not reachable")
                time.sleep(0.02)
        self.seq = 0
        self.fd = -1
        self.mm: Optional[mmap.mmap] = None
        self.size = 0
        self.prof = {"n": 0, "copy_in": 0.0, "round_trip": 0.0, "copy_out": 0.0} if PROFILE_PATH else None

    def _profile(self, t0: float, t1: float, t2: float, t3: float) -> None:
        p = self.prof
        p["n"] += 1
        p["copy_in"] += t1 - t0
        p["round_trip"] += t2 - t1
        p["copy_out"] += t3 - t2
        if p["n"] % 256 == 0:
            import json
            with open(PROFILE_PATH, "a") as f:
                f.write(json.dumps({"pid": os.getpid(), **p}) + "\n")

    def close(self) -> None:
        try:
            self.sock.close()
        finally:
            if self.mm is not None:
                self.mm.close()
            if self.fd >= 0:
                os.close(self.fd)
            self.mm, self.fd = None, -1

    def _call(self, kind: int, in_len: int, out_off: int, op, flip: bool, width: int = 0, height: int = 0,
              fds=None) -> int:
        self.seq += 1
        pkt = _REQ.pack(MAGIC, kind, self.seq, in_len, out_off, width, height, op.out_h, op.out_w,
                        op.crop_before_resize, op.filter, op.out_dtype, op.layout, int(bool(flip)), 0)
        if fds:
            socket.send_fds(self.sock, [pkt], fds)
        else:
            self.sock.send(pkt)
        rep = self.sock.recv(_REP.size)
        if len(rep) != _REP.size:
            raise ServiceError("the decode service closed the connection")
        seq, status, _ = _REP.unpack(rep)
        if seq != self.seq:
            raise ServiceError(f"decode service reply out of order ({seq} != {self.seq})")
        return status

    def _reserve(self, need: int) -> None:
        if need <= self.size:
            return
        size = _align(max(need, 2 * self.size, 8 << 20), 1 << 20)
        fd = os.memfd_create("sds_amd_region", os.MFD_CLOEXEC)
        os.ftruncate(fd, size)
        mm = mmap.mmap(fd, size)
        from ._lib import SdsjOp
        st = self._call(KIND_MAP, size, 0, SdsjOp(0, 0, 0, 0, 0, 0), False, fds=[fd])
        if st != OK:
            mm.close()
            os.close(fd)
            raise ServiceError(f"the decode service could not map the region (status {st})")
        if self.mm is not None:
            self.mm.close()
            os.close(self.fd)
        self.fd, self.mm, self.size = fd, mm, size

    def _result(self, status: int, off: int, op):
        if status != OK:
            return status, None
        dt = np.float32 if op.out_dtype == 1 else np.uint8
        shape = (op.out_h, op.out_w, 3) if op.layout == 1 else (3, op.out_h, op.out_w)
        arr = np.frombuffer(self.mm, dtype=dt, count=int(np.prod(shape)), offset=off).reshape(shape).copy()
        return status, arr

    def decode(self, data: bytes, op, flip: bool = False):
        """One JPEG -> (status, output array or None)."""
        t0 = time.perf_counter() if self.prof is not None else 0.0
        n = len(data)
        off = _align(n, 256)
        ob = op.out_h * op.out_w * 3 * (4 if op.out_dtype == 1 else 1)
        self._reserve(off + ob)
        self.mm[0:n] = data
        if self.prof is None:
            return self._result(self._call(KIND_DECODE, n, off, op, flip), off, op)
        t1 = time.perf_counter()
        st = self._call(KIND_DECODE, n, off, op, flip)
        t2 = time.perf_counter()
        r = self._result(st, off, op)
        self._profile(t0, t1, t2, time.perf_counter())
        return r

    def resize_frame(self, rgb: np.ndarray, op, flip: bool = False):
        """One HWC uint8 RGB frame (a sample PIL decoded) -> (status, output array or None)."""
        rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
        h, w = rgb.shape[:2]
        n = rgb.nbytes
        off = _align(n, 256)
        ob = op.out_h * op.out_w * 3 * (4 if op.out_dtype == 1 else 1)
        self._reserve(off + ob)
        self.mm[0:n] = rgb.reshape(-1).data
        return self._result(self._call(KIND_FRAME, n, off, op, flip, w, h), off, op)


_clients: dict[tuple[int, str], ServiceClient] = {}


def client(address: str) -> ServiceClient:
    key = (os.getpid(), address)
    c = _clients.get(key)
    if c is None:
        c = ServiceClient(address)
        _clients[key] = c
    return c


# ------------------------------------------------------------------------------------------------
# the service process
# ------------------------------------------------------------------------------------------------
def serve_main(argv=None) -> int:
    import argparse
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--address", required=True)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--parent", type=int, default=0)
    ap.add_argument("--engines", type=int, default=8)
    ap.add_argument("--max-batch", type=int, default=64)
    a = ap.parse_args(argv)
    sock = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    sock.bind(b"\0" + a.address.encode())
    sock.listen(1024)
    # idle until a worker connects (or the parent is gone): no GPU context for unused pipelines
    while True:
        if a.parent and os.getppid() != a.parent:
            return 0
        r, _, _ = select.select([sock], [], [], 1.0)
        if r:
            break
    import torch  # noqa: F401  (one HIP runtime in the process, as sds_amd/_lib.py explains)
    from . import _lib
    lib = _lib.load()
    sock.setblocking(False)
    cfg = _lib.SdsjServiceCfg(_lib.SDSJ_ABI_VERSION, a.device, a.engines, a.max_batch, sock.fileno(), a.parent)
    rc = lib.sdsj_service_serve(ctypes.byref(cfg))
    return 0 if rc == 0 else 1


if __name__ == "__main__":
    sys.exit(serve_main())
