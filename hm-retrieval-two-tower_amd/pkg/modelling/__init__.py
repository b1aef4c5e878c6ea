"""Two-tower modelling on MI355X (mirrors pkg.modelling of the reference)."""
