"""Host-side mirror of the reference's ``simulation/environment.py`` caller of the hot path."""
