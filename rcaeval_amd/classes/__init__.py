"""Data classes shared by the RCA heads and the RQ2 scorer (mirror of ``RCAEval/classes``)."""
