"""tone_amd -- MI355X-native streaming acoustic path for T-one (log-mel -> chunked Conformer -> CTC).

Drop-in for ``tone.onnx_wrapper.StreamingCTCModel`` (the acoustic model slot of
``tone.pipeline.StreamingCTCPipeline``), computed by hand-written CDNA4 HIP kernels in
``libtonehip.so`` behind a C ABI (``include/tonehip.h``).
"""

from . import config  # noqa: F401
from .state import flat_to_triton, triton_to_flat  # noqa: F401  (Triton cache_last_* interop)

__version__ = "0.1.0"


def __getattr__(name):  # lazy: importing the package must not require the HIP library
    if name in ("StreamingCTCModel", "ToneSession"):
        from . import model
        return getattr(model, name)
    raise AttributeError(name)
