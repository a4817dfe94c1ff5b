"""CPU oracle for the BigCodec path — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench cpu_baseline)."""
