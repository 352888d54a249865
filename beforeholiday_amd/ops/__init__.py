"""Op-level entry points, one module per reference extension (GPU: HIP, CPU: torch reference)."""
