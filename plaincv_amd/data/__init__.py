"""Input pipelines feeding the hot path: the LM's HF-arrow token datasets."""
