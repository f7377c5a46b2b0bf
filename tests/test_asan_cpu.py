"""Host code that parses untrusted bytes (sedx_wav_parse, csrc/wav_parse.cpp)
or walks index arithmetic (sedx_events, csrc/vad.cpp) built with
-fsanitize=address,undefined and run over a malformed-RIFF / edge-series
corpus (tests/native/asan_driver.cpp; SURVEY.md §5 "Race detection /
sanitizers": ASan build of the C++ host side).  CPU only."""
import os
import shutil
import subprocess

import pytest

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'sound-event-detection_amd')


@pytest.mark.skipif(shutil.which('g++') is None, reason='needs g++')
def test_asan_host_corpus():
    r = subprocess.run(['make', '-s', '-C', PKG, 'asan'], capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert 'clean' in out and 'ERROR: AddressSanitizer' not in out and 'runtime error' not in out, out[-4000:]
