"""Input shaping for the PC path (mirror of ``RCAEval/io``)."""
