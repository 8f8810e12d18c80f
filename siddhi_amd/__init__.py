"""siddhi_amd — MI355X execution path for Siddhi's windowed group-by aggregation."""
