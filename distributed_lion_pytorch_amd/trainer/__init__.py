"""AsyncTrainer family (HF Trainer integration) and the native training engine."""
