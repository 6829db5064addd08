"""pytest plugin: run the collected tests in reverse order, to catch tests
that depend on state an earlier test left in a module-scoped fixture.
Usage: python -m pytest -p pytest_reverse ... (with scripts/ on PYTHONPATH)."""


def pytest_collection_modifyitems(session, config, items):
    items.reverse()
