"""OpenAI-compatible serving of the Qwen3 decoder and the TTFT / per-token
latency benchmark (the reference's benchmarks/ai-benchmark, MI355X-native)."""
