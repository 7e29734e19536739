"""The driver's build check: __graft_entry__.build() compiles everything and loads the library."""


def test_build_compiles_and_loads():
    import __graft_entry__ as g
    g.build()
