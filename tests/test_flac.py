"""FLAC decoding of the example audio (t-one_amd/flac.py) and the committed PCM fixture."""

import hashlib
from pathlib import Path

import numpy as np
import pytest

from tone_amd.flac import FlacError, decode_flac, read_audio

GOLD = Path(__file__).parent / "golden" / "audio_short_pcm.npy"
REF = Path("/root/reference/tone/demo/audio_examples")
MD5 = "b55f6d6dc3d3cc96fa787957d788c736"     # STREAMINFO of audio_short.flac


def test_fixture_matches_streaminfo_md5():
    pcm = np.load(GOLD)
    assert pcm.dtype == np.int16 and pcm.shape == (50880,)
    assert hashlib.md5(pcm.astype("<i2").tobytes()).hexdigest() == MD5


@pytest.mark.skipif(not REF.exists(), reason="reference checkout not present (GPU box)")
@pytest.mark.parametrize("name", ["audio_short", "audio_long"])
def test_decoder_reproduces_md5_of_reference_files(name):
    pcm = read_audio(REF / f"{name}.flac")          # raises unless the STREAMINFO MD5 matches
    assert pcm.dtype == np.int32 and pcm.ndim == 1
    if name == "audio_short":
        np.testing.assert_array_equal(pcm, np.load(GOLD).astype(np.int32))


@pytest.mark.skipif(not REF.exists(), reason="reference checkout not present (GPU box)")
def test_corruption_is_detected():
    data = bytearray((REF / "audio_short.flac").read_bytes())
    data[20000] ^= 0x10
    with pytest.raises(FlacError):
        decode_flac(bytes(data))


def test_not_flac():
    with pytest.raises(FlacError):
        decode_flac(b"RIFF....WAVEfmt ")
