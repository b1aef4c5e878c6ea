from dataclasses import dataclass
from typing import Optional, Tuple


@dataclass
class Settings:
    """
    Settings for running the code end to end
    (reference: pkg/utils/settings.py:5-73; same fields and defaults).

    The *_tfrecord_path fields name the directories holding this framework's
    encoded shards (pkg.modelling.dataset), which replace TFRecords.
    """

    raw_data_filepath: str
    articles_data_filepath: str
    customers_data_filepath: str
    train_data_range: Tuple[str, str]
    test_data_range: Tuple[str, str]
    baseline_model_date_range: Tuple[str, str]
    date_col_name: str
    candidate_col_name: str
    candidate_tfrecord_path: str
    train_data_filepath: str
    test_data_filepath: str
    train_data_tfrecord_path: str
    test_data_tfrecord_path: str
    schema_filepath: str
    trained_model_path: str
    index_path: str
    baseline_index_path: str
    tensorboard_logs_dir: str = "./logs"
    max_tfrecord_rows: Optional[int] = None
