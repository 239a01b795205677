"""Drop-in mirrors of the reference's ``modules`` package (hot-path functions only)."""
