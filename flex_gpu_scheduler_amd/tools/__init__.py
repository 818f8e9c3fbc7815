"""Developer tools: native stress/TSan driver inputs, profiling helpers."""
