"""HL model interface (parity: ``/root/reference/iit/tasks/hl_model.py:4-7``)."""
from abc import ABC, abstractmethod


class HLModel(ABC):
    @abstractmethod
    def is_categorical(self) -> bool:
        """True -> cross-entropy / argmax metrics; False -> MSE / atol metrics."""
