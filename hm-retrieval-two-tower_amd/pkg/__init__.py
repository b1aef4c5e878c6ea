"""MI355X-native drop-in for the `pkg` package of
SelvinSelbaraju/hm-retrieval-two-tower (Schema / pkg.modelling API).

Logging is configured exactly as the reference does (pkg/__init__.py:3-6).
"""
import logging

logging.basicConfig(
    level=logging.INFO,
    format="%(asctime)s | %(levelname)s | %(name)s | %(message)s",
)

__version__ = "0.1.0"
