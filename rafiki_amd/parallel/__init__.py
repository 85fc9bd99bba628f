"""Distributed execution on one MI355X node: RCCL process groups, knob exchange, DP grad buckets."""
