"""empty (imported for side effects only by reference modules)"""
