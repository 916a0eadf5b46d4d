"""Import shim: exposes the ``t5gemma-tts_amd/`` directory as package ``t5gemma_tts_amd``.

The directory name carries a hyphen (repo layout contract), which Python cannot
import directly; defining ``__path__`` here turns this module into the package.
"""
import os as _os

__path__ = [_os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "t5gemma-tts_amd")]

from t5gemma_tts_amd.config import VoiceConfig, BackboneDims, named_config  # noqa: E402,F401
