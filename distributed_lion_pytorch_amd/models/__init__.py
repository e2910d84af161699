"""Native model families (GPT-2, Llama) with HF-compatible parameter names."""
