"""Host utilities: data, checkpoints, numerics helpers, timing."""
