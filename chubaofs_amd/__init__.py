"""chubaofs_amd -- MI355X-native erasure-coding engine for CubeFS blobstore.

Hot path: GF(2^8) Reed-Solomon / LRC Encode, Verify, Reconstruct behind the
blobstore/common/ec.Encoder interface, computed by hand-written gfx950 kernels
in csrc/ and exported through the C ABI in include/cfsec.h (libcfsec.so).

    codemode     -- Tactic table and stripe layouts (codemode.go mirror)
    reedsolomon  -- reedsolomon.Encoder seam (cfsec_rs_*)
    ec           -- ec.Encoder / lrcEncoder (cfsec_ec_*)
"""
from . import codemode  # noqa: F401  (pure host; no native code)

__all__ = ["codemode", "ec", "reedsolomon"]


def __getattr__(name):
    # ec / reedsolomon load libcfsec.so on import and raise if it is missing.
    if name in ("ec", "reedsolomon"):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
