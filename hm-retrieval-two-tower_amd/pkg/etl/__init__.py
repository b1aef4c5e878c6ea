"""ETL helpers (pandas only; outside the hot path)."""
