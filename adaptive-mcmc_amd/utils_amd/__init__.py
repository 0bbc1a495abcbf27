"""Drivers around the ARWMH kernel (reference python/utils/)."""
