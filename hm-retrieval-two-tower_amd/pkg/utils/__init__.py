"""Run settings (mirror of the reference pkg.utils)."""
