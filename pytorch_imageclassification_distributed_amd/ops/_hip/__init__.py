"""Parts of the HIP op layer; import them through ``ops.hip`` (the facade keeps flag writes coherent)."""
