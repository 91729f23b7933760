"""Test-only AV1 models (independent of csrc/codec/av1_*.h)."""
