from .trainer import ModelTrainer  # noqa: F401
