"""Scenario and parameter data the hot path's callers use (reference ``config/``)."""
