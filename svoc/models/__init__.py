"""Oracle-side models: synthetic oracle generators and the sentiment encoder path."""
