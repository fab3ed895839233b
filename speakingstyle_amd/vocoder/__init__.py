"""HiFi-GAN vocoder side: mel front-end with the HiFi-GAN framing, datasets (incl. the
fine-tuning mode on ground-truth-aligned mels), the DDP training loop with validation and
TensorBoard logging, and the inference entry points (wav -> mel -> wav, npy mel -> wav)."""
