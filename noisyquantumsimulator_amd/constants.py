"""Physical constants (SI) used by the host-side parameter derivation.

Values are CODATA constants with the exact float values the reference uses
(RG/constants.py:95-252), so derived Omega, V and rates agree bit-for-bit.
"""
import math

HBAR = 1.054571817e-34          # J s
C = 299792458.0                 # m/s (exact)
EPS0 = 8.8541878128e-12         # F/m
KB = 1.380649e-23               # J/K (exact)
MU_B = 9.2740100783e-24         # J/T
E_CHARGE = 1.602176634e-19      # C (exact)
RY_JOULES = 2.1798723611035e-18  # J
A0 = 5.29177210903e-11          # m
TWO_PI = 2.0 * math.pi
