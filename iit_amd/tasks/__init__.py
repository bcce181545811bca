"""Tasks: IOI, MNIST-PVR (synthetic digits), docstring, MQNLI."""
