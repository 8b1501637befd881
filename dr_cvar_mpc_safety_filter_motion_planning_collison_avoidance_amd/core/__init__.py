"""Host-side mirror of the reference's ``core/`` hot-path modules (same names, same semantics)."""
