"""Schema / Feature / config types (mirror of the reference's pkg.schema)."""
