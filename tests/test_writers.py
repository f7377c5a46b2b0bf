"""Output writers against the reference's formats:
 - write_xml: the SoundCaptionList document of pytorch/predict.py:264-268,
   :362-407 (name = file name without its directory, one SoundSegment per
   event with stime / dur / event attributes, dur = offset - onset as Python
   float arithmetic prints it, and the 'Others' segment when no event fired);
 - write_submission: utils/utilities.py:278-291, one tab-separated line per
   event, floats formatted by str.format.
CPU only (pure host code)."""
import os

from sedx import inference


def _events():
    return [{'filename': 'a.wav', 'onset': 0.4, 'offset': 10.0, 'event_label': 'Applause'},
            {'filename': 'a.wav', 'onset': 25.92, 'offset': 28.24,
             'event_label': 'Male_speech_man_speaking'},
            {'filename': 'a.wav', 'onset': 0.0, 'offset': 5.0, 'event_label': 'Siren'}]


def test_write_xml_events():
    xml = inference.write_xml('/data/in/IGFZfTxCc5I.wav', _events())
    lines = xml.split('\n')
    assert lines[0] == '<AudioDoc name="IGFZfTxCc5I.wav">'
    assert lines[1] == '\t<SoundCaptionList>'
    assert lines[2] == '\t\t<SoundSegment stime="0.4" dur="9.6" event="Applause">Applause</SoundSegment>'
    # 28.24 - 25.92 in binary floating point, printed the way str.format does
    assert lines[3] == ('\t\t<SoundSegment stime="25.92" dur="2.3199999999999967" '
                        'event="Male_speech_man_speaking">Male_speech_man_speaking</SoundSegment>')
    assert lines[4] == '\t\t<SoundSegment stime="0.0" dur="5.0" event="Siren">Siren</SoundSegment>'
    assert lines[5] == '\t</SoundCaptionList>'
    assert lines[6] == '</AudioDoc>' and len(lines) == 7      # no trailing newline


def test_write_xml_others():
    xml = inference.write_xml('clip.wav', [], start=5, end=10)
    assert xml == ('<AudioDoc name="clip.wav">\n\t<SoundCaptionList>\n'
                   '\t\t<SoundSegment stime="5" dur="5">Others</SoundSegment>\n'
                   '\t</SoundCaptionList>\n</AudioDoc>')


def test_write_submission(tmp_path):
    p = os.path.join(str(tmp_path), 'sub.tsv')
    inference.write_submission(_events(), p)
    with open(p) as f:
        got = f.read()
    assert got == ('a.wav\t0.4\t10.0\tApplause\n'
                   'a.wav\t25.92\t28.24\tMale_speech_man_speaking\n'
                   'a.wav\t0.0\t5.0\tSiren\n')


def test_events_to_writers_roundtrip():
    """events_from_framewise (host C++ vad) feeding both writers: onsets are
    frame / 100 as predict.py:110-114 computes them."""
    import numpy as np
    fw = np.zeros((1, 1000, 25), np.float32)
    fw[0, 120:480, 3] = 0.9           # Cheering
    ev = inference.events_from_framewise(fw, inference.DEFAULT_PREDICT_PARAMS, audio_name='x.wav')
    assert ev == [{'filename': 'x.wav', 'onset': 1.2, 'offset': 4.8, 'event_label': 'Cheering'}]
    xml = inference.write_xml('x.wav', ev)
    assert '<SoundSegment stime="1.2" dur="3.5999999999999996" event="Cheering">Cheering</SoundSegment>' in xml
