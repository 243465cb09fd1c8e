"""ctypes driver of the MATLAB MEX gateway (matlab/vo_mex.c) built against the minimal mx-API in
tests/mex_shim/ (test infrastructure; MATLAB is not installed in this pipeline).

`Mex(path).call('cmd', *args, nout=k)` does what MATLAB does for `[o1..ok] = vo_mex('cmd', ...)`:
numpy arguments become column-major mxArrays of the matching class, mexFunction runs, and the
outputs come back as numpy arrays (a gateway error raises MexError with MATLAB's identifier).
Every successful call is also checked for leaked mxMalloc blocks / arrays."""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent / "mex_shim"
FAKE = HERE / "build" / "libvo_mex_fake.so"
REAL = HERE / "build" / "libvo_mex.so"

# MATLAB mxClassID values (mex.h)
CLASS = {np.dtype(np.float64): 6, np.dtype(np.float32): 7, np.dtype(np.uint8): 9, np.dtype(np.int32): 12,
         np.dtype(np.uint32): 13, np.dtype(np.bool_): 3}
DTYPE = {v: k for k, v in CLASS.items()}


class MexError(RuntimeError):
    def __init__(self, ident: str, msg: str):
        super().__init__(f"{ident}: {msg}")
        self.ident = ident


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


class Mex:
    def __init__(self, path: Path):
        L = C.CDLL(str(path))
        vp = C.c_void_p
        L.shim_create.argtypes = [C.c_int, C.c_size_t, C.c_size_t, vp]
        L.shim_create.restype = vp
        L.shim_string.argtypes = [C.c_char_p]
        L.shim_string.restype = vp
        for f in ("shim_class",):
            getattr(L, f).argtypes = [vp]
        for f in ("shim_m", "shim_n"):
            getattr(L, f).argtypes = [vp]
            getattr(L, f).restype = C.c_size_t
        L.shim_data.argtypes = [vp]
        L.shim_data.restype = vp
        L.shim_destroy.argtypes = [vp]
        L.shim_destroy.restype = None
        L.shim_err_id.restype = C.c_char_p
        L.shim_err_msg.restype = C.c_char_p
        L.shim_call.argtypes = [C.c_int, C.POINTER(vp), C.c_int, C.POINTER(vp), C.POINTER(C.c_int)]
        L.shim_at_exit.restype = None
        self.L = L

    def _arr(self, a):
        if isinstance(a, str):
            return self.L.shim_string(a.encode())
        a = np.asarray(a)
        if a.ndim == 0:
            a = a.reshape(1, 1)
        if a.ndim != 2:
            raise ValueError("2-D arrays only")
        f = np.asfortranarray(a)                          # MATLAB storage: column-major
        return self.L.shim_create(CLASS[a.dtype], a.shape[0], a.shape[1], f.ctypes.data_as(C.c_void_p) if f.size else None)

    def _out(self, p):
        cls, m, n = self.L.shim_class(p), self.L.shim_m(p), self.L.shim_n(p)
        dt = DTYPE[cls]
        if m * n == 0:
            return np.zeros((m, n), dt)
        buf = (C.c_char * (m * n * dt.itemsize)).from_address(self.L.shim_data(p))
        return np.frombuffer(bytes(buf), dt).reshape(n, m).T.copy()

    def call(self, cmd: str, *args, nout: int = 1):
        ins = [self._arr(cmd)] + [self._arr(a) for a in args]
        prhs = (C.c_void_p * len(ins))(*ins)
        plhs = (C.c_void_p * max(nout, 1))()
        leaked = C.c_int(0)
        rc = self.L.shim_call(nout, plhs, len(ins), prhs, C.byref(leaked))
        for p in ins:
            self.L.shim_destroy(p)
        if rc:
            raise MexError(self.L.shim_err_id().decode(), self.L.shim_err_msg().decode())
        outs = []
        for k in range(nout):
            if plhs[k]:
                outs.append(self._out(plhs[k]))
                self.L.shim_destroy(plhs[k])
            else:
                outs.append(None)
        assert leaked.value == 0, f"vo_mex('{cmd}') leaked {leaked.value} mxMalloc blocks / arrays"
        return outs[0] if nout == 1 else tuple(outs)

    def at_exit(self):
        """MATLAB's `clear mex`: run the gateway's mexAtExit handler (releases its context)."""
        self.L.shim_at_exit()
