"""Mirror of the reference's `zombsole.gym` package (multi-agent surface)."""
