"""Docstring-completion HL task."""
from .docstring_hl import ArgMoverHead, Docstring_HL, InductionHead
