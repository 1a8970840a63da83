"""Causal LM family (mirrors models/LM/)."""
