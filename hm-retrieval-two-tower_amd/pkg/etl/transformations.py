"""DataFrame helpers used by the runners (mirror of
/root/reference/pkg/etl/transformations.py; pandas only, outside the hot path)."""
import logging
import os
from typing import Tuple

import pandas as pd

logger = logging.getLogger(__name__)


def date_filter(df: pd.DataFrame, df_name: str, date_col: str, date_range: Tuple[str, str]) -> pd.DataFrame:
    """Rows with date_range[0] <= df[date_col] <= date_range[1]."""
    logger.info(f"Creating df {df_name} from: {date_range[0]} to: {date_range[1]}")
    return df[(df[date_col] >= date_range[0]) & (df[date_col] <= date_range[1])]


def load_dataframe(path: str, df_name: str) -> pd.DataFrame:
    logger.info(f"Loading {df_name} from {path}")
    return pd.read_csv(path)


def save_dataframe(df: pd.DataFrame, df_name: str, date_col: str, path: str) -> None:
    logger.info(f"Saving {df_name} ({len(df)} rows) to {path}")
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    df.sort_values(date_col).to_csv(path, index=False)
