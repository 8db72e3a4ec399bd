from .base_tuner import BaseTuner
from .index_based_tuner import GridSearchTuner, RandomTuner
from .model_based_tuner import ModelBasedTuner

__all__ = ["BaseTuner", "GridSearchTuner", "RandomTuner", "ModelBasedTuner"]
