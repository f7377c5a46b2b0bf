"""sedx — MI355X-native inference path of yazdayy/sound-event-detection.

Public surface (mirrors the reference's hot-path API):
  sedx.models      Cnn_9layers_Gru_FrameAtt, Cnn_9layers_Transformer_FrameAtt (+ helpers)
  sedx.inference   predict_windows, inference_prob, gamma_features, events_from_framewise
  sedx.distributed clip sharding + framewise gather over RCCL
  sedx.synth       seeded synthetic weights / waveforms (bench, tests)
"""
__version__ = '0.1.0'
