"""Drop-in mirrors of the reference's ``apis`` package (hot-path classes only)."""
