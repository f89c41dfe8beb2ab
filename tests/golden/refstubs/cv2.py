"""empty stand-in (fixture generation only)"""
