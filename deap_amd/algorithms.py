"""Evolutionary loops that drive the GP evaluation hot path.

Behavioural restatement of the reference's ``deap/algorithms.py``.  Every loop
evaluates through ``toolbox.map(toolbox.evaluate, invalid_ind)`` — the call the
GPU evaluator intercepts (reference ``algorithms.py:150,172`` for ``eaSimple``,
``:301,:320`` for ``eaMuPlusLambda``, ``:399,:420`` for ``eaMuCommaLambda``).
The loops are unchanged; only the registered ``map``/``evaluate`` differ.
"""
import random

from . import tools

__all__ = ["varAnd", "varOr", "eaSimple", "eaMuPlusLambda",
           "eaMuCommaLambda", "eaGenerateUpdate"]


def _evaluate_invalid(population, toolbox):
    invalid = [ind for ind in population if not ind.fitness.valid]
    fitnesses = toolbox.map(toolbox.evaluate, invalid)
    for ind, fit in zip(invalid, fitnesses):
        ind.fitness.values = fit
    return len(invalid)


def varAnd(population, toolbox, cxpb, mutpb):
    """Clone, then crossover consecutive pairs with probability *cxpb*, then
    mutate each with probability *mutpb* (reference ``algorithms.py:33-82``)."""
    offspring = [toolbox.clone(ind) for ind in population]
    for i in range(1, len(offspring), 2):
        if random.random() < cxpb:
            offspring[i - 1], offspring[i] = toolbox.mate(offspring[i - 1],
                                                          offspring[i])
            del offspring[i - 1].fitness.values, offspring[i].fitness.values
    for i in range(len(offspring)):
        if random.random() < mutpb:
            offspring[i], = toolbox.mutate(offspring[i])
            del offspring[i].fitness.values
    return offspring


def eaSimple(population, toolbox, cxpb, mutpb, ngen, stats=None,
             halloffame=None, verbose=__debug__):
    """Generational EA (reference ``algorithms.py:85-189``)."""
    logbook = tools.Logbook()
    logbook.header = ["gen", "nevals"] + (stats.fields if stats else [])

    nevals = _evaluate_invalid(population, toolbox)
    if halloffame is not None:
        halloffame.update(population)
    record = stats.compile(population) if stats else {}
    logbook.record(gen=0, nevals=nevals, **record)
    if verbose:
        print(logbook.stream)

    for gen in range(1, ngen + 1):
        offspring = toolbox.select(population, len(population))
        offspring = varAnd(offspring, toolbox, cxpb, mutpb)
        nevals = _evaluate_invalid(offspring, toolbox)
        if halloffame is not None:
            halloffame.update(offspring)
        population[:] = offspring
        record = stats.compile(population) if stats else {}
        logbook.record(gen=gen, nevals=nevals, **record)
        if verbose:
            print(logbook.stream)
    return population, logbook


def varOr(population, toolbox, lambda_, cxpb, mutpb):
    """Produce *lambda_* children by crossover, mutation or reproduction
    (reference ``algorithms.py:192-245``)."""
    assert (cxpb + mutpb) <= 1.0, (
        "The sum of the crossover and mutation probabilities must be smaller "
        "or equal to 1.0.")
    offspring = []
    for _ in range(lambda_):
        op_choice = random.random()
        if op_choice < cxpb:
            ind1, ind2 = [toolbox.clone(i)
                          for i in random.sample(population, 2)]
            ind1, ind2 = toolbox.mate(ind1, ind2)
            del ind1.fitness.values
            offspring.append(ind1)
        elif op_choice < cxpb + mutpb:
            ind = toolbox.clone(random.choice(population))
            ind, = toolbox.mutate(ind)
            del ind.fitness.values
            offspring.append(ind)
        else:
            offspring.append(random.choice(population))
    return offspring


def _ea_mu_lambda(population, toolbox, mu, lambda_, cxpb, mutpb, ngen, stats,
                  halloffame, verbose, plus):
    logbook = tools.Logbook()
    logbook.header = ["gen", "nevals"] + (stats.fields if stats else [])
    nevals = _evaluate_invalid(population, toolbox)
    if halloffame is not None:
        halloffame.update(population)
    record = stats.compile(population) if stats is not None else {}
    logbook.record(gen=0, nevals=nevals, **record)
    if verbose:
        print(logbook.stream)
    for gen in range(1, ngen + 1):
        offspring = varOr(population, toolbox, lambda_, cxpb, mutpb)
        nevals = _evaluate_invalid(offspring, toolbox)
        if halloffame is not None:
            halloffame.update(offspring)
        pool = population + offspring if plus else offspring
        population[:] = toolbox.select(pool, mu)
        record = stats.compile(population) if stats is not None else {}
        logbook.record(gen=gen, nevals=nevals, **record)
        if verbose:
            print(logbook.stream)
    return population, logbook


def eaMuPlusLambda(population, toolbox, mu, lambda_, cxpb, mutpb, ngen,
                   stats=None, halloffame=None, verbose=__debug__):
    """(mu + lambda) EA (reference ``algorithms.py:248-337``)."""
    return _ea_mu_lambda(population, toolbox, mu, lambda_, cxpb, mutpb, ngen,
                         stats, halloffame, verbose, plus=True)


def eaMuCommaLambda(population, toolbox, mu, lambda_, cxpb, mutpb, ngen,
                    stats=None, halloffame=None, verbose=__debug__):
    """(mu , lambda) EA (reference ``algorithms.py:340-437``)."""
    assert lambda_ >= mu, "lambda must be greater or equal to mu."
    return _ea_mu_lambda(population, toolbox, mu, lambda_, cxpb, mutpb, ngen,
                         stats, halloffame, verbose, plus=False)


def eaGenerateUpdate(toolbox, ngen, halloffame=None, stats=None,
                     verbose=__debug__):
    """Ask-tell loop (reference ``algorithms.py:440-497``): each generation
    ``toolbox.generate()`` a population, evaluate it through
    ``toolbox.map`` (one GPU call with :func:`deap_amd.evaluator.gpu_map`),
    update the hall of fame, ``toolbox.update(population)``, record."""
    logbook = tools.Logbook()
    logbook.header = ["gen", "nevals"] + (stats.fields if stats else [])
    population = None
    for gen in range(ngen):
        population = toolbox.generate()
        for ind, fit in zip(population,
                            toolbox.map(toolbox.evaluate, population)):
            ind.fitness.values = fit
        if halloffame is not None:
            halloffame.update(population)
        toolbox.update(population)
        logbook.record(gen=gen, nevals=len(population),
                       **(stats.compile(population) if stats is not None
                          else {}))
        if verbose:
            print(logbook.stream)
    return population, logbook
