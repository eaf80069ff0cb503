"""Drop-in replacement of the reference's ``control`` package (control/MPC.py and friends)."""
