from dataclasses import dataclass
from typing import Any, Dict, Optional


@dataclass
class TrainingConfig:
    """
    Hyperparameters for training
    (reference: pkg/schema/training_config.py:5-39).

    Parameters
    ----------
    train_batch_size: int
        Number of rows in a single batch of train data.
    test_batch_size: int
        Number of rows in a single batch of test data.
    optimizer_name: str
        Name of the optimizer ("adagrad" or "adam").
    optimizer_kwargs: Dict[str, Any]
        Kwargs for the optimizer; must contain "learning_rate".
    candidate_batch_size: int
        Batch size for indexing candidates.
    shuffle_size: Optional[int]
        Shuffle buffer size. If None, don't shuffle.
    epochs: int
        Number of training rounds.
    candidate_prob_lookup: Optional[Dict[str, float]]
        Optional lookup (candidate id -> probability) for logQ correction.
    """

    train_batch_size: int
    test_batch_size: int
    optimizer_name: str
    optimizer_kwargs: Dict[str, Any]
    candidate_batch_size: int = 10000
    shuffle_size: Optional[int] = None
    epochs: int = 1
    candidate_prob_lookup: Optional[Dict[str, float]] = None
