"""Frozen hyper-parameters and the flat per-stream state layout of the T-one acoustic path.

Every constant here restates a reference default; the citations are relative to the
reference checkout (ToolsAiforia/T-one):

* feature front-end  -- ``tone/training/model_wrapper.py:28-35`` (sr 8000, win 0.02 s, hop 0.01 s,
  n_fft 160, 64 mels, pre-emphasis 0.97) and ``tone/nn/modules/feats.py:33-63``.
* encoder            -- ``tone/training/model_wrapper.py:37-75``.
* CTC head           -- ``tone/training/model_wrapper.py:76-115`` (34 labels + blank id 34).
* boundary constants -- ``tone/onnx_wrapper.py:30-34``.

The flat state order is the argument order of ``Tone.forward_for_export``
(``tone/nn/model.py:101-113``): preproc | mhsa | conv | mhsa_len | sub1 | sub2 | reduction.
The HF ``model.onnx`` that fixes the real order is not in the reference repository
(SURVEY.md 8b), so this order is the documented, reproducible choice; converters to the
Triton 5-tensor form live in :mod:`tone_amd.state`.
"""

from __future__ import annotations

# --- boundary constants (tone/onnx_wrapper.py:30-34) -------------------------------------
SAMPLE_RATE = 8000
MEAN_TIME_BIAS = 0.33
AUDIO_CHUNK_SAMPLES = 2400
FRAME_SIZE = 0.03
STATE_SIZE = 219729

# --- feature front-end (feats.py:33-63, model_wrapper.py:28-35) ---------------------------
WIN_LENGTH = 160
HOP_LENGTH = 80
N_FFT = 160
N_BINS = N_FFT // 2 + 1          # 81
N_MELS = 64
PREEMPH = 0.97
PREPROC_STATE = N_FFT - HOP_LENGTH   # 80 samples of left context (feats.py:58)
MEL_FRAMES = (AUDIO_CHUNK_SAMPLES + PREPROC_STATE - WIN_LENGTH) // HOP_LENGTH + 1  # 30
LOG_GUARD = 2.0 ** -24           # feats.py:19

# --- encoder (model_wrapper.py:37-75) ------------------------------------------------------
D_MODEL = 384
N_LAYERS = 16
N_HEADS = 8
D_HEAD = D_MODEL // N_HEADS      # 48
D_FF = 4 * D_MODEL               # 1536
ROPE_DIM = 32
ROPE_BASE = 10000.0
CONV_KERNEL = 31
CONV_STATE = CONV_KERNEL - 1     # 30 (conformer.py:99)
MHSA_STATELESS = 14              # layers >= 14 keep an MHSA input cache
MHSA_STATE = 30
CHUNK_FRAMES = 10                # acoustic frames per 300 ms chunk
REDUCTION_POS = 6
UPSAMPLE_POS = 14
REDUCTION_FACTOR = 2
REDUCTION_KERNEL = 3
RECOMPUTE_SCORES = (True, False, False, False, False, False, False,
                    True, False, False, False, False, False, False, True, True)

SUB_CH = (32, 64)
SUB_K = ((11, 21), (11, 11))
SUB_STRIDE = ((1, 1), (3, 1))
SUB1_STATE = SUB_K[0][0] - SUB_STRIDE[0][0]     # 10 time rows of normed features
SUB2_STATE = SUB_K[1][0] - SUB_STRIDE[1][0]     # 8 time rows of conv1 output
SUB1_F = N_MELS - SUB_K[0][1] + 1               # 44
SUB2_F = SUB1_F - SUB_K[1][1] + 1               # 34
SUB_OUT_IN = SUB_CH[1] * SUB2_F                 # 2176
RED_STATE = REDUCTION_KERNEL - REDUCTION_FACTOR  # 1

RMS_EPS = 1e-8      # submodules.py:28
LN_EPS = 1e-5       # nn.LayerNorm default (submodules.py:196-197)
BN_EPS = 1e-5       # nn.BatchNorm default

VOCAB = 35          # 34 labels + blank
BLANK_ID = 34
LABELS = "абвгдеёжзийклмнопрстуфхцчшщъыьэюя "   # tone/decoder.py:23


def layer_frames(layer: int) -> int:
    """Acoustic frames a layer sees per chunk: 10, or 5 inside the reduced block 7..14."""
    return CHUNK_FRAMES // REDUCTION_FACTOR if REDUCTION_POS < layer <= UPSAMPLE_POS else CHUNK_FRAMES


def mhsa_cache_rows(layer: int) -> int:
    """Rows of cached MHSA input a layer attends over (EncoderState.update_before_layer,
    conformer_blocks.py:147-148): 15 for layer 14 (reduced), 30 for layer 15, 0 otherwise."""
    if layer < MHSA_STATELESS:
        return 0
    return MHSA_STATE // REDUCTION_FACTOR if REDUCTION_POS < layer <= UPSAMPLE_POS else MHSA_STATE


# --- flat state layout, per stream, fp16 elements --------------------------------------------
N_MHSA_LAYERS = N_LAYERS - MHSA_STATELESS                       # 2
OFF_PREPROC = 0
OFF_MHSA = OFF_PREPROC + PREPROC_STATE                          # 80
OFF_CONV = OFF_MHSA + N_MHSA_LAYERS * MHSA_STATE * D_MODEL       # 23120
OFF_MHSA_LEN = OFF_CONV + N_LAYERS * D_MODEL * CONV_STATE       # 207440
OFF_SUB1 = OFF_MHSA_LEN + 1                                     # 207441
OFF_SUB2 = OFF_SUB1 + SUB1_STATE * N_MELS                       # 208081
OFF_RED = OFF_SUB2 + SUB_CH[0] * SUB2_STATE * SUB1_F            # 219345
STATE_END = OFF_RED + D_MODEL * RED_STATE                       # 219729
assert STATE_END == STATE_SIZE

STATE_SECTIONS = {
    # name: (offset, shape per stream)
    "preproc": (OFF_PREPROC, (PREPROC_STATE,)),
    "mhsa": (OFF_MHSA, (N_MHSA_LAYERS, MHSA_STATE, D_MODEL)),
    "conv": (OFF_CONV, (N_LAYERS, D_MODEL, CONV_STATE)),
    "mhsa_len": (OFF_MHSA_LEN, (1,)),
    "sub1": (OFF_SUB1, (1, SUB1_STATE, N_MELS)),
    "sub2": (OFF_SUB2, (SUB_CH[0], SUB2_STATE, SUB1_F)),
    "reduction": (OFF_RED, (D_MODEL, RED_STATE)),
}

# --- work per stream-chunk --------------------------------------
FLOP_PER_CHUNK_ENCODER_HEAD = 1_285_872_640
FLOP_PER_CHUNK_MEL = 1_870_000
FLOP_PER_CHUNK = FLOP_PER_CHUNK_ENCODER_HEAD + FLOP_PER_CHUNK_MEL
STATE_BYTES = 2 * STATE_SIZE
# algorithmic HBM bytes one stream-chunk moves at the boundary: state in + out, PCM in, logprobs out
IO_BYTES_PER_CHUNK = 2 * STATE_BYTES + 4 * 2400 + 4 * 10 * 35
