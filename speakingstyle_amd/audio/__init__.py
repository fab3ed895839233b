from . import io, mel, stft  # noqa: F401
