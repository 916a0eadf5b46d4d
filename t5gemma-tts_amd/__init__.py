"""MI355X-native T5Gemma-TTS generate() engine (package body; see ../t5gemma_tts_amd.py)."""
