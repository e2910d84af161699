"""Process-group bootstrap, vote exchange strategies and fault tolerance."""
