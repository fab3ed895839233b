"""speakingstyle_amd -- MI355X-native FastSpeech2 + speaking-style TTS framework.

Capabilities of lordzuko/SpeakingStyle (FastSpeech2 + FiLM reference encoder,
GST, word-level prosody control, HiFi-GAN) re-designed for AMD Instinct MI355X
(gfx950): channel-last bf16 activations, hand-written HIP/CDNA4 kernels for the
hot ops (``csrc/``), one process per GPU with RCCL gradient buckets.
"""
__version__ = "0.1.0"
