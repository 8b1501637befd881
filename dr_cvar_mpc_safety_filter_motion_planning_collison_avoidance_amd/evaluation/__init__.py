"""Timing-harness counterpart (evaluation/timing_analysis.py) for the GPU engine."""
