"""Decode the reference's example utterance (tone/demo/audio_examples/audio_short.flac: mono 8 kHz
16-bit, 50,880 samples) with tone_amd.flac and store the PCM as tests/golden/audio_short_pcm.npy.
The decoder verifies the result against the MD5 the encoder stored in the file's STREAMINFO
(b55f6d6dc3d3cc96fa787957d788c736), so the fixture is bit-exact with what the reference's
read_example_audio() (tone/demo/read_audio.py:17-53, miniaudio) returns for this file.
Run here (needs /root/reference); the fixture travels to the GPU box, the reference does not."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from tone_amd.flac import read_audio  # noqa: E402

SRC = Path("/root/reference/tone/demo/audio_examples/audio_short.flac")

if __name__ == "__main__":
    pcm = read_audio(SRC)
    out = Path(__file__).parent / "audio_short_pcm.npy"
    np.save(out, pcm.astype(np.int16))
    print(f"{out}: {pcm.shape[0]} samples, min {pcm.min()}, max {pcm.max()}")
