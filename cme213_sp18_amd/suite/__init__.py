"""HIP kernel suite covering the CME213 homework workloads."""
